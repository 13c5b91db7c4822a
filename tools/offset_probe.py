"""Does the repair array's placement relative to the received-source array change the decode apply's
time (two streams hitting the same HBM channels at the same time)?  The headline's apply (k16 e4 L1200,
2^20 blocks, packed output) with the repair array placed at several byte offsets inside one larger
allocation; offsets alternate over cycles.  Timing only, plus a check that every offset's recovered
rows equal offset 0's.
usage: python tools/offset_probe.py [--cycles=N]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import make_erasures  # noqa: E402
from pquic_amd import Engine  # noqa: E402

cycles = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--cycles=")), 5))
eng = Engine(0)
dev = torch.device("cuda:0")
nb, k, r, L, e = 1 << 20, 16, 4, 1200, 4
src = torch.empty((nb, k, L), dtype=torch.uint8, device=dev)
eng.synth_fill(src, src.numel(), 0x5EEDF3C0, 0)
OFFS = [0, 256, 4096, 65536, 1 << 20, (2 << 20) + 4096, 7 * 4096 + 1024]
big = torch.empty(nb * r * L + max(OFFS), dtype=torch.uint8, device=dev)
reps = {o: big[o: o + nb * r * L].view(nb, r, L) for o in OFFS}
work = src.clone()
sp, miss = make_erasures(torch, nb, k, e, 11, dev)
idx = (torch.arange(nb, device=dev).unsqueeze(1) * k + miss.to(dev)).reshape(-1)
work.view(nb * k, L)[idx] = 0xA5
rp = torch.zeros((nb, 2), dtype=torch.int64, device=dev)
rp[:, 0] = (1 << r) - 1
st = torch.empty(nb, dtype=torch.uint8, device=dev)
rec = torch.empty((nb, 2), dtype=torch.int64, device=dev)
ws = eng.alloc_workspace(nb, k, r)
eng.rlc_decode_plan(sp, rp, k, r, nb, ws)
out = torch.empty((nb, e, L), dtype=torch.uint8, device=dev)
ref = None
for o in OFFS:  # every placement holds the same repairs; its apply must give the same rows
    eng.rlc_encode(src, reps[o], k, r, L)
    eng.rlc_decode_apply_packed(work, reps[o], out, st, rec, k, r, L, nb, ws)
    torch.cuda.synchronize()
    if ref is None:
        ref = out.clone()
    assert torch.equal(out, ref), o
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
times = {o: [] for o in OFFS}
for _ in range(cycles):
    for o in OFFS:
        eng.rlc_encode(src, reps[o], k, r, L)  # the bench's order: the apply right after its encode
        ev[0].record()
        for _ in range(3):
            eng.rlc_decode_apply_packed(work, reps[o], out, st, rec, k, r, L, nb, ws)
        ev[1].record()
        torch.cuda.synchronize()
        times[o].append(ev[0].elapsed_time(ev[1]) / 3)
for o in OFFS:
    print(f"repair array at +{o:9d} B: apply {statistics.median(times[o]):.3f} ms (min {min(times[o]):.3f})",
          flush=True)
