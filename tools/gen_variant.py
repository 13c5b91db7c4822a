"""Build a generator variant of the engine for in-process A/B: regenerate bitslice_gen.h with the
given FEC_GEN_* settings into pquic_amd/lib/variants/<name>/ and build libpquic_fec.so there
against it (select it with ab_inproc.py "name:LIB=pquic_amd/lib/variants/<name>/libpquic_fec.so").
usage: python tools/gen_variant.py NAME [FEC_GEN_X=V ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pquic_amd import build as B  # noqa: E402

name, sets = sys.argv[1], sys.argv[2:]
vdir = os.path.join(B.LIBDIR, "variants", name)
os.makedirs(vdir, exist_ok=True)
hdr = os.path.join(vdir, "bitslice_gen.h")
env = dict(os.environ, FEC_GEN_OUT=hdr, **dict(s.split("=", 1) for s in sets))
subprocess.run([sys.executable, os.path.join(B.CSRC, "gen_bitslice.py")], env=env, check=True)
B.build(verbose=True, out=os.path.join(vdir, "libpquic_fec.so"), defines=[f'FEC_GEN_HDR="{hdr}"'])
