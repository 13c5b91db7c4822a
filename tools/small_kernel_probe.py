"""Where a one-block kernel's time goes: device time per launch (events around back-to-back
launches, so host launch cost is hidden) for one-block encodes and decodes of growing size, against a
16-byte fill as the empty-kernel floor.  The slope per coefficient tells apart the VALU cost of a case
(~30 ns) from a cold instruction fetch per case (L2 latency, a few hundred ns).
usage: python tools/small_kernel_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pquic_amd import Engine  # noqa: E402

eng = Engine(0)
dev = torch.device("cuda:0")
N = 400


def dev_us(fn, n=N):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


buf = torch.empty(1 << 16, dtype=torch.uint8, device=dev)
print(f"floor: 16-B fill {dev_us(lambda: eng.synth_fill(buf, 16, 1, 0)):.2f} us/launch")
L = 1200
for k, r in [(4, 1), (16, 1), (16, 2), (16, 4), (32, 4), (64, 4), (32, 8), (64, 8)]:
    for nb in (1, 8):
        src = torch.empty((nb, k, L), dtype=torch.uint8, device=dev)
        eng.synth_fill(src, src.numel(), 5, 0)
        rep = torch.empty((nb, r, L), dtype=torch.uint8, device=dev)
        t = dev_us(lambda: eng.rlc_encode(src, rep, k, r, L))
        print(f"encode k{k:<3d} r{r:<2d} blocks {nb}: {t:7.2f} us/launch, {t * 1e3 / (k * r):6.1f} ns per coefficient")
for k, r, e in [(16, 4, 1), (16, 4, 4), (32, 8, 8)]:
    src = torch.empty((1, k, L), dtype=torch.uint8, device=dev)
    eng.synth_fill(src, src.numel(), 5, 0)
    rep = torch.empty((1, r, L), dtype=torch.uint8, device=dev)
    eng.rlc_encode(src, rep, k, r, L)
    sp = torch.tensor([[((1 << k) - 1) & ~((1 << e) - 1), 0]], dtype=torch.int64, device=dev)
    rp = torch.tensor([[(1 << r) - 1, 0]], dtype=torch.int64, device=dev)
    st = torch.empty(1, dtype=torch.uint8, device=dev)
    rec = torch.empty((1, 2), dtype=torch.int64, device=dev)
    ws = eng.alloc_workspace(1, k, r)
    t = dev_us(lambda: eng.rlc_decode(src, rep, sp, rp, st, rec, k, r, L, workspace=ws))
    print(f"decode k{k:<3d} r{r:<2d} e{e:<2d} 1 block: {t:7.2f} us/launch")

# Small batches: blocks per wave-group shrink below min_groups groups (knob), A/B against the
# per-shape group sizes (min_groups=0).
print("batch sweep: us/launch with min_groups=0 (per-shape groups) -> default")
for k, r in [(16, 4), (32, 8), (64, 16)]:
    for nb in (8, 32, 128, 512, 2048, 8192):
        src = torch.empty((nb, k, L), dtype=torch.uint8, device=dev)
        eng.synth_fill(src, src.numel(), 5, 0)
        rep = torch.empty((nb, r, L), dtype=torch.uint8, device=dev)
        n = max(20, min(N, 20000 // nb))
        with eng.knob("min_groups", 0):
            t0 = dev_us(lambda: eng.rlc_encode(src, rep, k, r, L), n)
            ref = rep.clone()
        t1 = dev_us(lambda: eng.rlc_encode(src, rep, k, r, L), n)
        assert torch.equal(ref, rep)
        e = r
        sp = torch.zeros((nb, 2), dtype=torch.int64)
        sp[:, 0] = ((1 << k) - 1) & ~((1 << e) - 1) if k < 64 else -1 & ~((1 << e) - 1)
        sp = sp.to(dev)
        rp = torch.zeros((nb, 2), dtype=torch.int64)
        rp[:, 0] = (1 << r) - 1
        rp = rp.to(dev)
        st = torch.empty(nb, dtype=torch.uint8, device=dev)
        rec = torch.empty((nb, 2), dtype=torch.int64, device=dev)
        ws = eng.alloc_workspace(nb, k, r)
        with eng.knob("min_groups", 0):
            d0 = dev_us(lambda: eng.rlc_decode(src, rep, sp, rp, st, rec, k, r, L, workspace=ws), n)
        d1 = dev_us(lambda: eng.rlc_decode(src, rep, sp, rp, st, rec, k, r, L, workspace=ws), n)
        print(f"k{k:<3d} r{r:<2d} blocks {nb:5d}: encode {t0:8.1f} -> {t1:8.1f}   decode e{e} {d0:8.1f} -> {d1:8.1f}")
