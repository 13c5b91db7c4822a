"""In-process A/B of whole library builds (e.g. tools/build_at_commit.sh outputs) on the bench's data
path: k16 r4 encode and k16 e4 decode apply (2^20 blocks, random erasures, recovered rows at their
slots and packed), k32 r8 encode and k32 e8 decode apply (2^19 blocks).  Every build runs on the same
buffers; variants alternate over cycles; prints the median and min kernel time per (variant, case).
--check: before timing, every variant's packed apply (k16 e4, k32 e8) must give the first variant's statuses,
recovered masks and recovered rows (the rows of unknowns whose bit is set), byte for byte.
--k64: configs[4] too (k64 r16 L9000 encode and e16 packed apply, 2^16 blocks).  Knobs a variant sets are
restored to their values from before it ran (variants of one library share its knobs).
usage: python tools/lib_ab.py name=path.so[:knob=value,...] ... [--cycles=N] [--check] [--k64]"""
import ctypes as C
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import make_erasures  # noqa: E402
from pquic_amd import Engine  # noqa: E402

cycles = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--cycles=")), 5))
# name=path[:knob=value,...]: a build, optionally with knobs set while its cases run
variants, knobs = [], {}
for arg in (a for a in sys.argv[1:] if not a.startswith("--")):
    name, rest = arg.split("=", 1)
    path, _, kv = rest.partition(":")
    variants.append((name, path))
    knobs[name] = dict((x.split("=")[0], int(x.split("=")[1])) for x in kv.split(",") if x)
dev = torch.device("cuda:0")
eng0 = Engine(0)
engines = {n: Engine(0, lib_path=p) for n, p in variants}


def has_packed(e):
    try:
        e.lib.fecgpu_rlc_decode_apply_packed.argtypes = [C.c_void_p] * 3 + [C.c_uint64] + [C.c_uint32] * 3 + \
            [C.c_void_p] * 3 + [C.c_size_t, C.c_void_p]
        return True
    except AttributeError:
        return False


def dec_setup(k, r, e, L, nb, seed):
    src = torch.empty((nb, k, L), dtype=torch.uint8, device=dev)
    eng0.synth_fill(src, src.numel(), seed, 0)
    rep = torch.empty((nb, r, L), dtype=torch.uint8, device=dev)
    eng0.rlc_encode(src, rep, k, r, L)
    work = src.clone()
    sp, miss = make_erasures(torch, nb, k, e, 11, dev)
    idx = (torch.arange(nb, device=dev).unsqueeze(1) * k + miss.to(dev)).reshape(-1)
    work.view(nb * k, L)[idx] = 0xA5
    rp = torch.zeros((nb, 2), dtype=torch.int64, device=dev)
    rp[:, 0] = (1 << r) - 1
    st = torch.empty(nb, dtype=torch.uint8, device=dev)
    rec = torch.empty((nb, 2), dtype=torch.int64, device=dev)
    ws = eng0.alloc_workspace(nb, k, r)
    eng0.rlc_decode_plan(sp, rp, k, r, nb, ws)
    rec_pk = torch.empty((nb, min(k, r), L), dtype=torch.uint8, device=dev)
    return dict(src=src, rep=rep, work=work, st=st, rec=rec, ws=ws, rec_pk=rec_pk, k=k, r=r, L=L, nb=nb,
                miss=miss.sort(dim=1).values.to(dev))


cases = []
d16 = dec_setup(16, 4, 4, 1200, 1 << 20, 0x5EEDF3C0)
rec_to = torch.empty_like(d16["src"])
cases.append(("enc k16r4", lambda e: e.rlc_encode(d16["src"], d16["rep"], 16, 4, 1200)))
cases.append(("app_to k16e4", lambda e: e.rlc_decode_apply_to(d16["work"], d16["rep"], rec_to, d16["st"], d16["rec"],
                                                               16, 4, 1200, d16["nb"], d16["ws"])))
cases.append(("app_pk k16e4", lambda e: e.rlc_decode_apply_packed(d16["work"], d16["rep"], d16["rec_pk"], d16["st"],
                                                                   d16["rec"], 16, 4, 1200, d16["nb"], d16["ws"])))
d32 = dec_setup(32, 8, 8, 1200, 1 << 19, 0x5EEDF3C1)
cases.append(("enc k32r8", lambda e: e.rlc_encode(d32["src"], d32["rep"], 32, 8, 1200)))
cases.append(("app_pk k32e8", lambda e: e.rlc_decode_apply_packed(d32["work"], d32["rep"], d32["rec_pk"], d32["st"],
                                                                   d32["rec"], 32, 8, 1200, d32["nb"], d32["ws"])))
checks = [(d16, 4), (d32, 8)]
if "--k64" in sys.argv:
    d64 = dec_setup(64, 16, 16, 9000, 1 << 16, 0x5EEDF3C2)
    cases.append(("enc k64r16", lambda e: e.rlc_encode(d64["src"], d64["rep"], 64, 16, 9000)))
    cases.append(("app_pk k64e16", lambda e: e.rlc_decode_apply_packed(d64["work"], d64["rep"], d64["rec_pk"],
                                                                        d64["st"], d64["rec"], 64, 16, 9000,
                                                                        d64["nb"], d64["ws"])))
    checks.append((d64, 16))


def set_knobs(e, kv):
    """sets a variant's knobs; returns their previous values"""
    old = {k: e.get_knob(k) for k in kv}
    for k, v in kv.items():
        e.set_knob(k, v)
    return old


if "--check" in sys.argv:
    for d, e_ in checks:
        ref = None
        for name, _ in variants:
            e = engines[name]
            old = set_knobs(e, knobs[name])
            d["rec_pk"].fill_(0x5A)
            d["st"].fill_(0xEE)
            e.rlc_decode_apply_packed(d["work"], d["rep"], d["rec_pk"], d["st"], d["rec"], d["k"], d["r"], d["L"],
                                      d["nb"], d["ws"])
            torch.cuda.synchronize()
            set_knobs(e, old)
            # rows of unknowns whose recovered bit is set (the u-th missing source of the block)
            bits = ((d["rec"][:, 0:1] >> d["miss"].clamp(max=63)) & 1).bool() & (d["miss"] < 64)
            got = (d["st"].clone(), d["rec"].clone(), d["rec_pk"][:, :e_][bits].clone())
            if ref is None:
                ref = got
                assert (got[0] == 0).sum().item() > d["nb"] * 0.9
            else:
                ok = all(torch.equal(a, b) for a, b in zip(got, ref))
                print(f"check k{d['k']} e{e_}: {name} {'equal to' if ok else 'DIFFERS from'} {variants[0][0]}", flush=True)
                if not ok:
                    sys.exit(1)
times = {}
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for cyc in range(cycles):
    for name, _ in variants:
        e = engines[name]
        old = set_knobs(e, knobs[name])
        for cname, fn in cases:
            if cname.startswith("app_pk") and not has_packed(e):
                continue
            fn(e)
            ev[0].record()
            for _ in range(3):
                fn(e)
            ev[1].record()
            torch.cuda.synchronize()
            times.setdefault((name, cname), []).append(ev[0].elapsed_time(ev[1]) / 3)
        set_knobs(e, old)
print(f"{'variant':10s} " + " ".join(f"{c:>18s}" for c, _ in cases) + "   (median ms; min)")
for name, _ in variants:
    cells = []
    for cname, _ in cases:
        t = times.get((name, cname))
        cells.append(f"{statistics.median(t):8.3f}/{min(t):7.3f}" if t else f"{'-':>16s}")
    print(f"{name:10s} " + " ".join(f"{x:>18s}" for x in cells), flush=True)
