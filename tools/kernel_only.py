"""Run one data-path kernel configuration repeatedly (for rocprofv3 counter passes).
usage: python tools/kernel_only.py {enc,dec} K R [blocks] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pquic_amd import Engine  # noqa: E402

mode, k, r = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
nb = int(sys.argv[4]) if len(sys.argv) > 4 else (1 << 20)
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
L = int(os.environ.get("FEC_L", "1200"))
eng = Engine(0)
dev = torch.device("cuda:0")
src = torch.empty((nb, k, L), dtype=torch.uint8, device=dev)
eng.synth_fill(src, src.numel(), 1, 0)
rep = torch.empty((nb, r, L), dtype=torch.uint8, device=dev)
eng.rlc_encode(src, rep, k, r, L)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
if mode == "enc":
    for _ in range(reps):
        eng.rlc_encode(src, rep, k, r, L)
else:
    e = min(k, r)
    sp = torch.zeros((nb, 2), dtype=torch.int64, device=dev)
    sp[:, 0] = ((1 << k) - 1) & ~((1 << e) - 1) if k < 64 else -1 << e
    rp = torch.zeros((nb, 2), dtype=torch.int64, device=dev)
    rp[:, 0] = (1 << r) - 1
    st = torch.empty(nb, dtype=torch.uint8, device=dev)
    rec = torch.empty((nb, 2), dtype=torch.int64, device=dev)
    ws = eng.alloc_workspace(nb, k, r)
    for _ in range(reps):
        eng.rlc_decode(src, rep, sp, rp, st, rec, k, r, L, workspace=ws)
ev[1].record()
torch.cuda.synchronize()
print(f"done {mode} k={k} r={r} L={L} blocks={nb}: {ev[0].elapsed_time(ev[1]) / reps:.3f} ms per call")
