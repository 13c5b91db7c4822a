"""Is the batching adapter's one-sender rate a property of the process it runs in?  bench.py's
batch_saturated leg runs in a process that imported torch first; tools/sender_phase_probe.py runs in a
fresh one.  torch's wheel bundles its own HIP and HSA runtimes under the same sonames as /opt/rocm's, so
whichever loads first serves the engine library too.  Modes (one per process):
  fresh    -- the engine library first: /opt/rocm's runtime
  torchrt  -- torch's bundled libhsa-runtime64 / libamdhip64 preloaded (RTLD_GLOBAL), torch not imported
  torch    -- `import torch` first (bench.py's order)
  torch1   -- as torch, then torch.set_num_threads(1)
  bench    -- as torch, then bench.py's prelude one piece at a time, a rate after each: the engine and its
              headline tensors (2^20 blocks) with an encode + decode, then the PCIe legs
Prints the median of `runs` batch_saturated runs and the HIP runtime file actually mapped.
usage: python tools/batch_context_probe.py MODE [runs]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
mode = sys.argv[1]
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
if mode == "torchrt":
    import importlib.util
    tl = os.path.join(os.path.dirname(importlib.util.find_spec("torch").origin), "lib")
    for n in ("libhsa-runtime64.so", "libamdhip64.so"):
        C.CDLL(os.path.join(tl, n), mode=C.RTLD_GLOBAL)
elif mode.startswith("torch"):
    import torch
    if mode == "torch1":
        torch.set_num_threads(1)
if mode == "bench":
    import torch
lib = C.CDLL(os.path.join(ROOT, "tools", "libbatchload.so"))
lib.bl_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.c_uint, C.c_uint, C.c_int,
                       C.c_double, C.c_int, C.POINTER(C.c_double)]
lib.bl_set_inflight.argtypes = [C.c_int]
lib.bl_set_inflight(3)


def rate(tag):
    res = []
    for _ in range(runs):
        out = (C.c_double * 8)()
        rc = lib.bl_run(0, 16, 4, 1200, 64, 200000, 2048, 2000, 2, 0.0, 3, out)
        res.append(out[0] if rc == 0 else -1.0)
    res.sort()
    rt = sorted({ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln})
    print(f"{tag}: batch_saturated {res[len(res) // 2]:.2f} GiB/s, runs {['%.2f' % x for x in res]}; HIP runtime "
          f"{rt}", flush=True)


rate(mode)
if mode == "bench":
    sys.path.insert(0, ROOT)
    import argparse
    import bench
    from pquic_amd import Engine
    eng = Engine(0)
    rate("bench: engine created")
    dev = torch.device("cuda:0")
    nb, k, r, e, L = 1 << 20, 16, 4, 4, 1200
    src = torch.empty((nb, k, L), dtype=torch.uint8, device=dev)
    eng.synth_fill(src, src.numel(), 1, 0)
    rep = torch.empty((nb, r, L), dtype=torch.uint8, device=dev)
    work = src.clone()
    sp, miss = bench.make_erasures(torch, nb, k, e, 11, dev)
    rp = torch.zeros((nb, 2), dtype=torch.int64, device=dev)
    rp[:, 0] = (1 << r) - 1
    st = torch.empty(nb, dtype=torch.uint8, device=dev)
    rec = torch.empty((nb, 2), dtype=torch.int64, device=dev)
    ws = eng.alloc_workspace(nb, k, r)
    dst = torch.empty((nb, e, L), dtype=torch.uint8, device=dev)
    for _ in range(3):
        eng.rlc_encode(src, rep, k, r, L)
        eng.rlc_decode_stages(work, rep, sp, rp, st, rec, k, r, L, nb, ws, dst=dst, packed=True)
    torch.cuda.synchronize()
    rate("bench: headline tensors and kernels")
    args = argparse.Namespace(k=16, r=4, symbol=1200, erasures=4, blocks=nb)
    legs = bench.pcie_legs(torch, args, dev)
    rate("bench: after the PCIe legs")
    del src, rep, work, dst
    torch.cuda.empty_cache()
    rate("bench: device tensors freed")
