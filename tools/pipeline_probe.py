"""Headline workload (k=16 r=4, 4 erasures, 2^20 blocks, 1200-B symbols) as a serial step against a
pipelined one.  serial: the bench's step (plan on a second stream beside the encode, then the apply,
which reads the encode's repairs).  pipelined: a sender and a receiver are independent, so step s encodes
batch s on one stream while batch s-1 (its repairs and plan double-buffered) is applied on another.
Same buffers and kernels; prints median ms per step.  usage: python tools/pipeline_probe.py [--cycles=N]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import make_erasures  # noqa: E402
from pquic_amd import Engine  # noqa: E402

cycles = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--cycles=")), 5))
reps = 10
eng = Engine(0)
dev = torch.device("cuda:0")
nb, k, r, L, e = 1 << 20, 16, 4, 1200, 4
src = torch.empty((nb, k, L), dtype=torch.uint8, device=dev)
eng.synth_fill(src, src.numel(), 0x5EEDF3C0, 0)
rep = [torch.empty((nb, r, L), dtype=torch.uint8, device=dev) for _ in range(2)]
sp, miss = make_erasures(torch, nb, k, e, 11, dev)
work = src.clone()
idx = (torch.arange(nb, device=dev).unsqueeze(1) * k + miss.to(dev)).reshape(-1)
work.view(nb * k, L)[idx] = 0xA5
rp = torch.zeros((nb, 2), dtype=torch.int64, device=dev)
rp[:, 0] = (1 << r) - 1
st = torch.empty(nb, dtype=torch.uint8, device=dev)
rec = torch.empty((nb, 2), dtype=torch.int64, device=dev)
ws = [eng.alloc_workspace(nb, k, r) for _ in range(2)]
rows = torch.empty((nb, min(k, r), L), dtype=torch.uint8, device=dev)
main = torch.cuda.current_stream(dev)
plan_s = torch.cuda.Stream(dev)
app_s = torch.cuda.Stream(dev)
ev = lambda: torch.cuda.Event()  # noqa: E731
applied = [ev(), ev()]
for x in applied:
    x.record(main)


def serial(s):
    go = ev()
    go.record(main)
    plan_s.wait_event(go)
    eng.rlc_decode_plan(sp, rp, k, r, nb, ws[0], stream=plan_s)
    planned = ev()
    planned.record(plan_s)
    eng.rlc_encode(src, rep[0], k, r, L)
    main.wait_event(planned)
    eng.rlc_decode_apply_packed(work, rep[0], rows, st, rec, k, r, L, nb, ws[0])


enc_done, planned2 = [ev(), ev()], [ev(), ev()]


def pipelined(s):
    b = s % 2
    plan_s.wait_event(applied[b])  # ws[b] and rep[b] were last read by the apply of batch s - 2
    eng.rlc_decode_plan(sp, rp, k, r, nb, ws[b], stream=plan_s)
    planned2[b].record(plan_s)
    main.wait_event(applied[b])
    eng.rlc_encode(src, rep[b], k, r, L)
    enc_done[b].record(main)
    if s > 0:  # batch s - 1
        a = 1 - b
        app_s.wait_event(enc_done[a])
        app_s.wait_event(planned2[a])
        eng.rlc_decode_apply_packed(work, rep[a], rows, st, rec, k, r, L, nb, ws[a], stream=app_s)
        applied[a].record(app_s)


serial(0)
torch.cuda.synchronize()
ok0 = st == 0
for s in range(3):
    pipelined(s)
torch.cuda.synchronize()
assert bool(((st == 0) == ok0).all()), "pipelined decode status differs"
times = {"serial": [], "pipelined": []}
t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(cycles):
    for name, fn in (("serial", serial), ("pipelined", pipelined)):
        fn(0)
        fn(1)
        torch.cuda.synchronize()
        t0.record(main)
        plan_s.wait_event(t0)
        app_s.wait_event(t0)
        for s in range(2, 2 + reps):
            fn(s)
        done = ev()
        done.record(app_s)
        main.wait_event(done)
        t1.record(main)
        torch.cuda.synchronize()
        times[name].append(t0.elapsed_time(t1) / reps)
for name, t in times.items():
    print(f"{name:10s} step {statistics.median(t):7.3f} ms (min {min(t):.3f})  "
          f"{nb * k * L / 2**30 / (statistics.median(t) * 1e-3):8.1f} GiB/s", flush=True)
