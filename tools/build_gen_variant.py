"""Build the engine with the data-path bodies generated under other FEC_GEN_* settings (A/B builds for
tools/lib_ab.py / tools/ab_inproc.py): copies pquic_amd/ and include/ to a scratch tree, regenerates
bitslice_gen.h there with the given environment, and builds pquic_amd/lib/variants/NAME/libpquic_fec.so.
usage: python tools/build_gen_variant.py NAME VAR=VALUE ... [-DMACRO=VALUE ...]"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
name = sys.argv[1]
env = dict(os.environ)
defines = []
for a in sys.argv[2:]:
    if a.startswith("-D"):
        defines.append(a[2:])
    else:
        k, v = a.split("=", 1)
        env[k] = v
tmp = tempfile.mkdtemp(prefix=f"genvar_{name}_")
try:
    for d in ("pquic_amd", "include"):
        shutil.copytree(os.path.join(ROOT, d), os.path.join(tmp, d),
                        ignore=shutil.ignore_patterns("lib", "__pycache__"))
    csrc = os.path.join(tmp, "pquic_amd", "csrc")
    env["FEC_GEN_OUT"] = os.path.join(csrc, "bitslice_gen.h")
    subprocess.run([sys.executable, os.path.join(csrc, "gen_bitslice.py")], env=env, check=True)
    out = os.path.join(ROOT, "pquic_amd", "lib", "variants", name, "libpquic_fec.so")
    code = (f"import sys; sys.path.insert(0, {tmp!r}); from pquic_amd import build as b; "
            f"b.build(out={out!r}, defines={defines!r}, verbose=True)")
    subprocess.run([sys.executable, "-c", code], check=True, cwd=tmp)
finally:
    shutil.rmtree(tmp, ignore_errors=True)
