"""In-process A/B of whole library builds on the XOR scheme legs (bench.py xor_leg shape: k=4, 1200-B
symbols, 2^22 blocks, one source erased per block): encode and decode kernel time, same buffers,
variants alternating.  usage: python tools/xor_ab.py name=path.so ... [--cycles=N]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pquic_amd import Engine  # noqa: E402

cycles = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--cycles=")), 5))
variants = [tuple(a.split("=", 1)) for a in sys.argv[1:] if not a.startswith("--")]
dev = torch.device("cuda:0")
engines = {n: Engine(0, lib_path=p) for n, p in variants}
k, L, nb = 4, 1200, 1 << 22
g = torch.Generator(device=dev).manual_seed(7)
src = torch.randint(0, 256, (nb, k, L), dtype=torch.uint8, device=dev, generator=g)
rep = torch.empty((nb, L), dtype=torch.uint8, device=dev)
miss = torch.randint(0, k, (nb,), device=dev, generator=g)
sp = torch.zeros((nb, 2), dtype=torch.int64, device=dev)
sp[:, 0] = ((1 << k) - 1) ^ (1 << miss)
rp = torch.ones((nb, 2), dtype=torch.int64, device=dev)
rp[:, 1] = 0
st = torch.empty(nb, dtype=torch.uint8, device=dev)
rec = torch.empty((nb, 2), dtype=torch.int64, device=dev)
work = src.clone()
work[torch.arange(nb, device=dev), miss] = 0
dst = torch.empty((nb, L), dtype=torch.uint8, device=dev)
CASES = ("enc", "dec", "dto") if all(hasattr(e.lib, "fecgpu_xor_decode_to") for e in engines.values()) else ("enc", "dec")
times = {(n, c): [] for n, _ in variants for c in CASES}
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for n, _ in variants:  # warm-up and check
    e = engines[n]
    e.xor_encode(src, rep, k, L)
    w = work.clone()
    e.xor_decode(w, rep, sp, rp, st, rec, k, L)
    torch.cuda.synchronize()
    assert bool((st == 0).all()) and bool((w == src).all()), f"{n}: decode did not restore the sources"
    del w
for _ in range(cycles):
    for n, _ in variants:
        e = engines[n]
        for c in CASES:
            ev[0].record()
            if c == "enc":
                e.xor_encode(src, rep, k, L)
            elif c == "dto":  # recovered symbols into rows of their own
                e.xor_decode_to(work, rep, dst, sp, rp, st, rec, k, L)
            else:
                e.xor_decode(work, rep, sp, rp, st, rec, k, L)
            ev[1].record()
            torch.cuda.synchronize()
            times[(n, c)].append(ev[0].elapsed_time(ev[1]))
print(f"{'variant':12s} " + " ".join(f"{'xor ' + c + ' k4':>18s}" for c in CASES) +
      "   (median ms / min; 2^22 blocks, L=1200; dto = recovered rows to their own buffer)")
for n, _ in variants:
    print(f"{n:12s} " + " ".join(f"{statistics.median(times[(n, c)]):8.3f}/{min(times[(n, c)]):8.3f}" for c in CASES))
