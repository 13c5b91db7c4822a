"""Step-schedule probe for the headline workload (k=16 r=4, 4 erasures, 2^20 blocks): the decode's
plan stage needs only the presence masks and the block numbers, not the encode's output, so it
can run on a second (high-priority) stream beside the encode.  Alternates the serial step
(encode -> plan -> apply on one stream) with the overlapped one (the bench's schedule) and, third, a
pipelined one in which the apply decodes the previous step's repairs (a second repair buffer) on the
side stream while the encode writes this step's: encode and apply run at the same time, as a
sender's encodes and a receiver's decodes would.  Every schedule uses the bench's packed apply; prints
median step times.  usage: python tools/overlap_probe.py [--cycles N] [--reps R]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pquic_amd import Engine  # noqa: E402

cycles = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--cycles=")), 5))
reps = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--reps=")), 10))
eng = Engine(0)
dev = torch.device("cuda:0")
nb, k, r, L, e = 1 << 20, 16, 4, 1200, 4
src = torch.empty((nb, k, L), dtype=torch.uint8, device=dev)
eng.synth_fill(src, src.numel(), 0x5EEDF3C0, 0)
rep = torch.empty((nb, r, L), dtype=torch.uint8, device=dev)
rep2 = torch.empty_like(rep)
work = src.clone()
dst = torch.empty((nb, e, L), dtype=torch.uint8, device=dev)
g = torch.Generator(device="cpu").manual_seed(11)
miss = torch.stack([torch.randperm(k, generator=g)[:e] for _ in range(1024)])  # 1024 patterns, cycled
miss = miss.repeat(nb // 1024, 1)
sp = torch.zeros((nb, 2), dtype=torch.int64)
sp[:, 0] = ((1 << k) - 1) - (1 << miss).sum(1)
sp = sp.to(dev)
rp = torch.zeros((nb, 2), dtype=torch.int64, device=dev)
rp[:, 0] = (1 << r) - 1
st = torch.empty(nb, dtype=torch.uint8, device=dev)
rec = torch.empty((nb, 2), dtype=torch.int64, device=dev)
ws = eng.alloc_workspace(nb, k, r)
main = torch.cuda.current_stream(dev)
side = torch.cuda.Stream(dev, priority=-1)
plan_done = torch.cuda.Event()
apply_done = torch.cuda.Event()
apply_done.record(main)


def serial():
    eng.rlc_encode(src, rep, k, r, L)
    eng.rlc_decode_plan(sp, rp, k, r, nb, ws, stream=main)
    eng.rlc_decode_apply_packed(work, rep, dst, st, rec, k, r, L, nb, ws, stream=main)


def overlapped():
    side.wait_event(apply_done)  # the previous step's apply still reads the workspace
    eng.rlc_decode_plan(sp, rp, k, r, nb, ws, stream=side)
    plan_done.record(side)
    eng.rlc_encode(src, rep, k, r, L)
    main.wait_event(plan_done)
    eng.rlc_decode_apply_packed(work, rep, dst, st, rec, k, r, L, nb, ws, stream=main)
    apply_done.record(main)


enc_done = torch.cuda.Event()
bufs = [rep, rep2]


def pipelined():
    """side: plan + apply of the repairs the previous step encoded; main: this step's encode into the
    other buffer (it waits for the apply that read that buffer two steps ago)"""
    old, new = bufs
    side.wait_event(enc_done)  # the previous step's encode wrote `old`
    eng.rlc_decode_plan(sp, rp, k, r, nb, ws, stream=side)
    eng.rlc_decode_apply_packed(work, old, dst, st, rec, k, r, L, nb, ws, stream=side)
    apply_done.record(side)
    eng.rlc_encode(src, new, k, r, L)
    enc_done.record(main)
    main.wait_event(apply_done)  # the step ends when both have
    bufs.reverse()


eng.rlc_encode(src, rep2, k, r, L)
enc_done.record(main)
idx = (torch.arange(nb, device=dev).unsqueeze(1) * k + miss.sort(dim=1).values.to(dev))
for fn in (serial, overlapped, pipelined, pipelined):  # every schedule restores the sources
    dst.fill_(0)
    torch.cuda.synchronize()  # the side stream's apply must not start before the fill
    fn()
    torch.cuda.synchronize()
    ok = (st == 0).nonzero().squeeze(1)
    assert bool((dst[ok] == src.view(nb * k, L)[idx[ok]].view(-1, e, L)).all()), fn.__name__
times = {"serial": [], "overlapped": [], "pipelined": []}
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for _ in range(cycles):
    for name, fn in (("serial", serial), ("overlapped", overlapped), ("pipelined", pipelined)):
        fn()
        torch.cuda.synchronize()
        ev[0].record(main)
        side.wait_event(ev[0])  # nothing of the timed steps starts before ev[0]
        for _ in range(reps):
            fn()
        ev[1].record(main)
        torch.cuda.synchronize()
        times[name].append(ev[0].elapsed_time(ev[1]) / reps)
for name, t in times.items():
    print(f"{name:12s} step {statistics.median(t):7.3f} ms (min {min(t):.3f})  "
          f"{2 * nb * k * L / 2**30 / (statistics.median(t) * 1e-3):8.1f} GiB/s (encode + decode payload)")
