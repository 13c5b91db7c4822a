"""One-block RLC decode (k16 e4, 1200-B symbols) timed by events, device-resident buffers vs
page-locked host buffers through the host path (zero copy, the synchronous hook's route), to split
the hook's kernel time into compute and PCIe round trips.  usage: python tools/small_decode_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pquic_amd import Engine, HostPath  # noqa: E402

eng = Engine(0)
dev = torch.device("cuda:0")
k, r, L, n = 16, 4, 1200, 2000
src = torch.empty((1, k, L), dtype=torch.uint8, device=dev)
eng.synth_fill(src, src.numel(), 5, 0)
rep = torch.empty((1, r, L), dtype=torch.uint8, device=dev)
eng.rlc_encode(src, rep, k, r, L)
sp = torch.tensor([[((1 << k) - 1) & ~0xF, 0]], dtype=torch.int64, device=dev)
rp = torch.tensor([[(1 << r) - 1, 0]], dtype=torch.int64, device=dev)
st = torch.empty(1, dtype=torch.uint8, device=dev)
rec = torch.empty((1, 2), dtype=torch.int64, device=dev)
ws = eng.alloc_workspace(1, k, r)


def lat(fn):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2] * 1e6


print(f"device-resident, 1 block decode + sync: p50 {lat(lambda: eng.rlc_decode(src, rep, sp, rp, st, rec, k, r, L, workspace=ws)):.1f} us")
print(f"device-resident, 1 block encode + sync: p50 {lat(lambda: eng.rlc_encode(src, rep, k, r, L)):.1f} us")
hp = HostPath(0, 1, 1 << 20)
pin = lambda shape, dt: torch.empty(shape, dtype=dt, pin_memory=True)  # noqa: E731
hsrc, hrep = pin((1, k, L), torch.uint8), pin((1, r, L), torch.uint8)
hsrc.copy_(src.cpu())
hrep.copy_(rep.cpu())
hsp, hrp = pin((1, 2), torch.int64), pin((1, 2), torch.int64)
hsp.copy_(sp.cpu())
hrp.copy_(rp.cpu())
hst, hrec = pin(1, torch.uint8), pin((1, 2), torch.int64)
hseeds = pin((1, r), torch.int32)
hseeds.copy_(torch.arange(r, dtype=torch.int32).view(1, r))
print(f"page-locked host path, 1 block decode: p50 {lat(lambda: hp.rlc_decode_seeded(hsrc, hrep, hseeds, hsp, hrp, hst, hrec, 1, k, r, L)):.1f} us")
print(f"page-locked host path, 1 block encode: p50 {lat(lambda: hp.rlc_encode(hsrc, hrep, 1, k, r, L)):.1f} us")
print(f"empty sync: p50 {lat(lambda: None):.1f} us")
