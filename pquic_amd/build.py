"""Build the engine in-tree: pquic_amd/lib/libpquic_fec.so (hipcc, gfx950 only).

The .so holds the HIP kernels, the fecgpu_* C ABI (include/fecgpu.h) and the C protoop
adapters (include/pquic_fec_protoops.h).  Built with explicit hipcc/gcc command lines so
the artefact lives in the tree and travels to the GPU box with the snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libpquic_fec.so")
ARCH = "gfx950"


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build pquic_amd)")


def _run(cmd, **kw):
    r = subprocess.run(cmd, capture_output=True, text=True, **kw)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("build step failed: " + " ".join(cmd))
    return r


def sources():
    hip = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))
    c = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".c"))
    hdr = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h"))
    inc = os.path.join(ROOT, "include")
    hdr += sorted(os.path.join(inc, f) for f in os.listdir(inc) if f.endswith(".h"))
    return hip, c, hdr


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    hip, c, hdr = sources()
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(f) <= t for f in hip + c + hdr + [__file__])


def build(force: bool = False, verbose: bool = False, out: str | None = None, defines=()) -> str:
    """Build LIB (or, for A/B experiments, `out` with extra -D `defines`)."""
    if out is None and not defines and not force and up_to_date():
        return LIB
    target = out or LIB
    os.makedirs(LIBDIR, exist_ok=True)
    os.makedirs(os.path.dirname(target), exist_ok=True)
    hip, c, _ = sources()
    hipcc = _hipcc()
    objs = []
    odir = os.path.dirname(target)  # objects next to the target: variant builds may run in parallel
    inc = ["-I" + os.path.join(ROOT, "include"), "-I" + CSRC]
    for src in c:  # host C: the protoop adapters stay C (reference language)
        obj = os.path.join(odir, os.path.basename(src) + ".o")
        _run(["gcc", "-std=c11", "-O2", "-g", "-fPIC", "-Wall", "-Wextra", "-c", src, "-o", obj] + inc)
        objs.append(obj)
    for src in hip:
        obj = os.path.join(odir, os.path.basename(src) + ".o")
        _run([hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", obj] + inc +
             ["-D" + d for d in defines])
        objs.append(obj)
    tmp = target + ".tmp"
    _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs)
    os.replace(tmp, target)
    for o in objs:
        os.remove(o)
    if verbose:
        print("built", target)
    return target


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
