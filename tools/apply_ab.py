"""In-process A/B of the k16 e4 decode apply on the bench's buffers (random erasures, 2^20 blocks):
recovered rows at their src-layout slots (apply_to) or packed per block (apply_packed), at several
group caps (knob group; 0 = the default of 8 blocks).  Alternates variants over cycles; prints the
median and min apply time per variant.
usage: python tools/apply_ab.py [--cycles=N]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import make_erasures  # noqa: E402
from pquic_amd import Engine  # noqa: E402

cycles = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--cycles=")), 5))
nb, k, r, e, L = 1 << 20, 16, 4, 4, 1200
dev = torch.device("cuda:0")
eng = Engine(0)
src = torch.empty((nb, k, L), dtype=torch.uint8, device=dev)
eng.synth_fill(src, src.numel(), 0x5EEDF3C0, 0)
rep = torch.empty((nb, r, L), dtype=torch.uint8, device=dev)
eng.rlc_encode(src, rep, k, r, L)
work = src.clone()
sp, miss = make_erasures(torch, nb, k, e, 11, dev)
idx = (torch.arange(nb, device=dev).unsqueeze(1) * k + miss.to(dev)).reshape(-1)
work.view(nb * k, L)[idx] = 0xA5
rp = torch.zeros((nb, 2), dtype=torch.int64, device=dev)
rp[:, 0] = (1 << r) - 1
status = torch.empty(nb, dtype=torch.uint8, device=dev)
recovered = torch.empty((nb, 2), dtype=torch.int64, device=dev)
ws = eng.alloc_workspace(nb, k, r)
rec_to = torch.empty_like(src)
rec_pk = torch.empty((nb, min(k, r), L), dtype=torch.uint8, device=dev)
eng.rlc_decode_plan(sp, rp, k, r, nb, ws)
variants = [("to G8", "to", 0), ("packed G8", "pk", 0), ("packed G16", "pk", 16), ("packed G4", "pk", 4),
            ("to G16", "to", 16)]
if "--small-groups" in sys.argv:
    variants += [("packed G2", "pk", 2), ("packed G1", "pk", 1), ("to G2", "to", 2)]


def run(kind):
    if kind == "to":
        eng.rlc_decode_apply_to(work, rep, rec_to, status, recovered, k, r, L, nb, ws)
    else:
        eng.rlc_decode_apply_packed(work, rep, rec_pk, status, recovered, k, r, L, nb, ws)


# correctness gate: the packed rows equal the src-layout rows of the same unknowns
run("to")
run("pk")
torch.cuda.synchronize()
ok = status == 0
ms = miss.sort(dim=1).values.to(dev)
rows_to = rec_to.view(nb * k, L)[(torch.arange(nb, device=dev).unsqueeze(1) * k + ms).reshape(-1)].view(nb, e, L)
assert bool((rows_to[ok] == rec_pk[ok, :e]).all()), "packed rows differ from apply_to rows"
assert bool((rec_pk[ok, :e] == src.view(nb * k, L)[(torch.arange(nb, device=dev).unsqueeze(1) * k + ms)
                                                    .reshape(-1)].view(nb, e, L)[ok]).all()), "packed rows wrong"
times = {v[0]: [] for v in variants}
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for cyc in range(cycles):
    for name, kind, g in variants:
        eng.set_knob("group", g)
        run(kind)
        ev[0].record()
        for _ in range(5):
            run(kind)
        ev[1].record()
        torch.cuda.synchronize()
        times[name].append(ev[0].elapsed_time(ev[1]) / 5)
eng.set_knob("group", 0)
n_rec = int(ok.sum())
for name, _, _ in variants:
    t = times[name]
    gbs = (k + e) * L * n_rec / (statistics.median(t) * 1e-3) / 1e9
    print(f"{name:12s} median {statistics.median(t):7.3f} ms  min {min(t):7.3f}  ({gbs:7.1f} GB/s, {gbs / 8000:.3f} of 8 TB/s)",
          flush=True)
