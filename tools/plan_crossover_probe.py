"""Decode plan kernel time per launch: the wave plan (a wave per block, row-parallel elimination;
knob plan=1 in LDS, plan=5 in registers where the system fits) against the automatic choice
(lane-parallel plans: reg / tile / lane above the wave-plan threshold), over batch sizes, to place
the crossover.  usage: python tools/plan_crossover_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pquic_amd import Engine  # noqa: E402

eng = Engine(0)
dev = torch.device("cuda:0")


def dev_us(fn, n):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


for k, r, e in [(16, 4, 4), (16, 4, 1), (32, 8, 8), (32, 8, 2), (64, 16, 16), (64, 16, 4)]:
    for nb in (65, 256, 1024, 2048, 4096, 8192, 16384, 65536):
        g = torch.Generator().manual_seed(nb + k)
        sp = torch.zeros((nb, 2), dtype=torch.int64)
        full = (1 << k) - 1
        for b in range(nb):
            miss = torch.randperm(k, generator=g)[:e].tolist()
            m = full
            for j in miss:
                m &= ~(1 << j)
            sp[b, 0] = m - (1 << 64) if m >= (1 << 63) else m
        rp = torch.zeros((nb, 2), dtype=torch.int64)
        rp[:, 0] = (1 << r) - 1
        sp, rp = sp.to(dev), rp.to(dev)
        ws = eng.alloc_workspace(nb, k, r)
        n = max(5, min(200, 200000 // nb))
        with eng.knob("plan", 1):
            tw = dev_us(lambda: eng.rlc_decode_plan(sp, rp, k, r, nb, ws), n)
            wsw = ws.clone()
        with eng.knob("plan", 5):
            tr = dev_us(lambda: eng.rlc_decode_plan(sp, rp, k, r, nb, ws), n)
        ta = dev_us(lambda: eng.rlc_decode_plan(sp, rp, k, r, nb, ws), n)
        print(f"k{k:<3d} r{r:<2d} e{e:<2d} blocks {nb:6d}: wave {tw:9.1f} us   wave-reg {tr:9.1f} us   "
              f"auto {ta:9.1f} us", flush=True)
