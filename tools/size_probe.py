"""k32 r8 encode time per block against the batch size (2^18 .. 2^21 blocks): does the bench leg's
footprint (2^21 blocks = 100 GB of rows) cost per-block time?  Buffers of the largest size, the
smaller batches run on their prefixes; sizes alternate over cycles.
usage: python tools/size_probe.py [--cycles=N]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pquic_amd import Engine  # noqa: E402

cycles = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--cycles=")), 4))
eng = Engine(0)
dev = torch.device("cuda:0")
k, r, L, NB = 32, 8, 1200, 1 << 21
src = torch.empty((NB, k, L), dtype=torch.uint8, device=dev)
eng.synth_fill(src, src.numel(), 0x5EEDF3C0, 0)
rep = torch.empty((NB, r, L), dtype=torch.uint8, device=dev)
sizes = [1 << 18, 1 << 19, 1 << 20, 1 << 21]
times = {n: [] for n in sizes}
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for _ in range(cycles):
    for n in sizes:
        reps = max(2, (1 << 22) // n)
        eng.rlc_encode(src, rep, k, r, L, nblocks=n)
        ev[0].record()
        for _ in range(reps):
            eng.rlc_encode(src, rep, k, r, L, nblocks=n)
        ev[1].record()
        torch.cuda.synchronize()
        times[n].append(ev[0].elapsed_time(ev[1]) / reps)
for n in sizes:
    t = statistics.median(times[n])
    print(f"k32 r8 encode {n:8d} blocks: {t:8.3f} ms  {t / n * 1e6:7.2f} ns/block  "
          f"{(k + r) * L * n / (t * 1e-3) / 1e9:7.1f} GB/s", flush=True)
