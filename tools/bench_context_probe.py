"""Why does the bench's k16 encode / decode apply run slower than the same kernels in
tools/ab_inproc.py on the same box?  Allocates the bench's buffers (bench.py main: src, rep, work,
rec_rows, workspace) and times, with HIP events per kernel:
  enc-b2b   5 encodes back to back
  app-b2b   5 decode applies (recovered rows to rec_rows) back to back, after one plan
  step      5 bench steps (encode, plan, apply) -- the bench's sequence
  step-sync the same with a device synchronisation between the kernels
  enc-fresh encode into a freshly allocated repair buffer
usage: python tools/bench_context_probe.py [--inplace] [--blocks N]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import make_erasures  # noqa: E402
from pquic_amd import Engine  # noqa: E402

nb = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--blocks=")), 1 << 20))
k, r, e, L = 16, 4, 4, 1200
dev = torch.device("cuda:0")
eng = Engine(0)
src = torch.empty((nb, k, L), dtype=torch.uint8, device=dev)
eng.synth_fill(src, src.numel(), 0x5EEDF3C0, 0)
rep = torch.empty((nb, r, L), dtype=torch.uint8, device=dev)
work = torch.empty_like(src)
sp, miss = make_erasures(torch, nb, k, e, 11, dev)
rp = torch.zeros((nb, 2), dtype=torch.int64, device=dev)
rp[:, 0] = (1 << r) - 1
status = torch.empty(nb, dtype=torch.uint8, device=dev)
recovered = torch.empty((nb, 2), dtype=torch.int64, device=dev)
ws = eng.alloc_workspace(nb, k, r)
work.copy_(src)
idx = (torch.arange(nb, device=dev).unsqueeze(1) * k + miss.to(dev)).reshape(-1)
work.view(nb * k, L)[idx] = 0xA5
rec_rows = torch.empty_like(src)
dst = None if "--inplace" in sys.argv else rec_rows


def ev():
    return torch.cuda.Event(enable_timing=True)


def enc(out=rep):
    eng.rlc_encode(src, out, k, r, L)


def plan():
    eng.rlc_decode_plan(sp, rp, k, r, nb, ws)


def app():
    if dst is None:
        eng.rlc_decode_apply(work, rep, status, recovered, k, r, L, nb, ws)
    else:
        eng.rlc_decode_apply_to(work, rep, dst, status, recovered, k, r, L, nb, ws)


def timed(fns, sync=False):
    """run fns in order; per-fn elapsed ms (HIP events around each)"""
    if sync:
        out = []
        for f in fns:
            a, b = ev(), ev()
            a.record()
            f()
            b.record()
            torch.cuda.synchronize()
            out.append(a.elapsed_time(b))
        return out
    es = [ev() for _ in range(len(fns) + 1)]
    for i, f in enumerate(fns):
        es[i].record()  # also the end of fn i - 1
        f()
    es[-1].record()
    torch.cuda.synchronize()
    return [es[i].elapsed_time(es[i + 1]) for i in range(len(fns))]


enc(); plan(); app(); torch.cuda.synchronize()
res = {}
for cyc in range(3):
    t = timed([enc] * 5)
    res.setdefault("enc-b2b", []).extend(t[1:])
    plan()
    t = timed([app] * 5)
    res.setdefault("app-b2b", []).extend(t[1:])
    t = timed([enc, plan, app] * 5)
    res.setdefault("step:enc", []).extend(t[3::3])
    res.setdefault("step:app", []).extend(t[5::3])
    t = timed([enc, plan, app] * 3, sync=True)
    res.setdefault("step-sync:enc", []).extend(t[3::3])
    res.setdefault("step-sync:app", []).extend(t[5::3])
    fresh = torch.empty((nb, r, L), dtype=torch.uint8, device=dev)
    t = timed([lambda: enc(fresh)] * 3)
    res.setdefault("enc-fresh-rep", []).extend(t[1:])
    del fresh
    t = timed([enc, app] * 4)  # no plan between (plan unchanged)
    res.setdefault("enc-app:enc", []).extend(t[2::2])
    res.setdefault("enc-app:app", []).extend(t[3::2])
for kk, v in res.items():
    print(f"{kk:16s} median {statistics.median(v):7.3f} ms  min {min(v):7.3f}  max {max(v):7.3f}  (n={len(v)})",
          flush=True)
