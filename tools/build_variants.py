"""Build A/B variants of libpquic_fec.so under pquic_amd/lib/variants/<name>/ (select one at run
time with PQUIC_AMD_LIB=...).  usage: python tools/build_variants.py name=DEF1,DEF2 ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pquic_amd import build as B  # noqa: E402

for spec in sys.argv[1:]:
    name, _, defs = spec.partition("=")
    out = os.path.join(B.LIBDIR, "variants", name, "libpquic_fec.so")
    B.build(verbose=True, out=out, defines=[d for d in defs.split(",") if d])
