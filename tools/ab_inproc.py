"""In-process A/B of engine knobs (fecgpu_set_knob; the FECGPU_* environment names are accepted
and mapped to knob names), so every variant runs on the same buffers in the same process: alternates variants for several cycles and
prints median kernel times.  Removes the process-to-process variance (buffer placement) that
dominates whole-bench A/B runs.
A variant may also name another build of the library: "name:LIB=pquic_amd/lib/variants/X/libpquic_fec.so"
(loaded side by side under its own handle).
usage: python tools/ab_inproc.py "name:VAR=VAL,VAR=VAL" ... [--cycles N] [--reps R] [--case=mode:k:r:nblocks:L ...]
[--only: drop the three default cases]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pquic_amd import Engine  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
cycles = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--cycles=")), 5))
reps = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--reps=")), 5))
variants = []
for spec in args or ["base"]:
    name, _, env = spec.partition(":")
    kvs = {}
    last = None
    for piece in env.split(","):  # a piece without "=" continues the previous value ("A=8,2")
        if "=" in piece:
            last, v = piece.split("=", 1)
            kvs[last] = v
        elif piece and last:
            kvs[last] += "," + piece
    variants.append((name, kvs))
PLAN = {"wave": 1, "lane": 2, "reg": 3, "tile": 4}


def to_knobs(env):
    """{knob name: int} from a variant's VAR=VAL pairs (knob names or FECGPU_* environment names)."""
    out = {}
    for kk, vv in env.items():
        if kk == "LIB":
            continue
        if kk == "FECGPU_ENC_TILE":
            a, b = vv.split(",")
            out["enc_tile_rt"], out["enc_tile_waves"] = int(a), int(b)
        elif kk == "FECGPU_PLAN":
            out["plan"] = PLAN.get(vv, 0)
        elif kk.startswith("FECGPU_"):
            out[kk[len("FECGPU_"):].lower()] = int(vv)
        else:
            out[kk] = int(vv)
    return out


knobs = sorted({k for _, e in variants for k in to_knobs(e)})

eng0 = Engine(0)
engines = {name: (Engine(0, lib_path=e["LIB"]) if "LIB" in e else eng0) for name, e in variants}
eng = eng0
dev = torch.device("cuda:0")
L = 1200


def setup(k, r, nb, e, L):
    src = torch.empty((nb, k, L), dtype=torch.uint8, device=dev)
    eng.synth_fill(src, src.numel(), 1, 0)
    rep = torch.empty((nb, r, L), dtype=torch.uint8, device=dev)
    eng.rlc_encode(src, rep, k, r, L)
    sp = torch.zeros((nb, 2), dtype=torch.int64, device=dev)
    sp[:, 0] = (((1 << k) - 1) & ~((1 << e) - 1)) if k < 63 else -(1 << e)
    sp[1::2, 0] = (((1 << k) - 1) & ~((1 << e) << 1)) if k < 63 else sp[1::2, 0]  # vary the erased slot
    rp = torch.zeros((nb, 2), dtype=torch.int64, device=dev)
    rp[:, 0] = (1 << r) - 1
    st = torch.empty(nb, dtype=torch.uint8, device=dev)
    rec = torch.empty((nb, 2), dtype=torch.int64, device=dev)
    ws = eng.alloc_workspace(nb, k, r)
    return src, rep, sp, rp, st, rec, ws


cases = []
DST = torch.empty(((1 << 20), 16, 1200), dtype=torch.uint8, device=dev) if "--apply-to" in sys.argv else None
FRAMES = torch.empty(((1 << 20) * 4 * 1216,), dtype=torch.uint8, device=dev) if "--frames" in sys.argv else None
CASES = [(16, 4, 1 << 20, "enc", 1200), (16, 4, 1 << 20, "dec", 1200), (32, 8, 1 << 20, "enc", 1200)]
if "--wide" in sys.argv:  # also the r >= 8 decode and configs[4] (jumbo symbols)
    CASES += [(32, 8, 1 << 19, "dec", 1200), (64, 16, 1 << 15, "enc", 9000), (64, 16, 1 << 15, "dec", 9000)]
if "--xor" in sys.argv:  # the XOR scheme (configs[0]'s) at GPU scale
    CASES += [(4, 1, 1 << 22, "xenc", 1200), (4, 1, 1 << 22, "xdec", 1200)]
if "--apply-to" in sys.argv:  # decode with the recovered rows written to a separate buffer
    CASES += [(16, 4, 1 << 20, "decto", 1200)]
if "--frames" in sys.argv:  # repair symbols -> FEC frames in 1216-B slots (the bench's frames leg)
    CASES += [(16, 4, 1 << 20, "frames", 1200)]
for spec in (a.split("=", 1)[1] for a in sys.argv if a.startswith("--case=")):  # mode:k:r:nblocks:L
    m, kk, rr, nn, ll = spec.split(":")
    CASES.append((int(kk), int(rr), int(nn), m, int(ll)))
if "--only" in sys.argv:
    CASES = CASES[3:]
for (k, r, nb, mode, L) in CASES:
    if mode.startswith("win"):  # window encode, mode "win<step>": nb windows over one symbol stream
        step = int(mode[3:])
        sym = torch.empty((((nb - 1) * step + k), L), dtype=torch.uint8, device=dev)
        eng.synth_fill(sym, sym.numel(), 3, 0)
        wrep = torch.empty((nb, r, L), dtype=torch.uint8, device=dev)
        cases.append((f"win s{step} k{k} r{r}" + ("" if L == 1200 else f" L{L}"), k, r, nb, mode, L,
                      (sym, wrep, None, None, None, None, None)))
        continue
    bufs = setup(k, r, nb, min(k, r), L)
    label = f"{mode} k{k} r{r}" + ("" if L == 1200 else f" L{L}")
    if any(c[0] == label for c in cases):  # the same shape at another batch size: labels (and the
        label += f" 2^{nb.bit_length() - 1}"  # digests and times keyed by them) must stay distinct
    cases.append((label, k, r, nb, mode, L, bufs))


def run(case, eng):
    _, k, r, nb, mode, L, (src, rep, sp, rp, st, rec, ws) = case
    if mode == "enc":
        eng.rlc_encode(src, rep, k, r, L)
    elif mode.startswith("win"):
        eng.rlc_window_encode(src, rep, nb, int(mode[3:]), k, r, L)
    elif mode == "xenc":
        eng.xor_encode(src, rep, k, L)
    elif mode == "xdec":
        eng.xor_decode(src, rep, sp, rp, st, rec, k, L)
    elif mode == "decto":
        eng.rlc_decode_plan(sp, rp, k, r, nb, ws)
        eng.rlc_decode_apply_to(src, rep, DST, st, rec, k, r, L, nb, ws)
    elif mode == "frames":
        eng.write_repair_frames(rep, FRAMES, nb, r, L, L, 1216, k, r)
    else:
        eng.rlc_decode(src, rep, sp, rp, st, rec, k, r, L, workspace=ws)


defaults = {(name, kn): engines[name].get_knob(kn) for name, _ in variants for kn in knobs}
times = {(v[0], c[0]): [] for v in variants for c in cases}
digests = {}
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for cyc in range(cycles):
    for name, env in variants:
        e = engines[name]
        want = to_knobs(env)
        for kn in knobs:  # unset knobs return to their defaults
            e.set_knob(kn, want.get(kn, defaults[(name, kn)]))
        for c in cases:
            run(c, e)  # warm
            if c[4] == "enc" or c[4].startswith("win"):  # every variant must produce the same repair bytes
                rep = c[6][1]
                sub = rep[::61].contiguous().view(torch.int32).view(-1).to(torch.int64)
                h = (sub * (torch.arange(sub.numel(), device=dev) % 65521 + 1)).sum().item()
                ref = digests.setdefault(c[0], h)
                if h != ref:
                    print(f"MISMATCH {name} {c[0]}", flush=True)
            ev[0].record()
            for _ in range(reps):
                run(c, e)
            ev[1].record()
            torch.cuda.synchronize()
            times[(name, c[0])].append(ev[0].elapsed_time(ev[1]) / reps)
print(f"{'variant':24s} " + " ".join(f"{c[0]:>16s}" for c in cases) + "   (median ms over cycles; min)")
for name, _ in variants:
    cells = []
    for c in cases:
        t = times[(name, c[0])]
        cells.append(f"{statistics.median(t):7.3f}/{min(t):6.3f}")
    print(f"{name:24s} " + " ".join(f"{x:>16s}" for x in cells))
