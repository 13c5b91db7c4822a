"""Where one sender thread's time goes at the saturated generate rate (tools/batch_load.c bl_run with
per-connection arenas, batches of 2048, 3 in flight -- the bench leg's setting): per block, the caller's
nanoseconds inside pquic_fec_batch_generate (submission: the protocol operation's allocations, queueing),
inside completions (poll: attach, done, the harness's frees), waiting for a free slot, and the rest (the
harness building its blocks), next to the batcher's engine- and stager-thread time.
Options (A/B in one process, the settings alternating run by run):
  --pf 0,8,16        completion prefetch distances (PQUIC_FEC_BATCH_PREFETCH, read per batcher)
  --lib a.so,b.so    load-generator builds (e.g. one built with -DBL_OLD_LAYOUT)
  --recover          the receiver (bl_run_recover, 4 erasures) instead of the sender
  --profile HZ       sample the sender thread's instruction address HZ times a second over the measured
                     passes (bl_set_sampling) and print where its time goes, per function and per line
usage: python tools/sender_phase_probe.py [runs] [--pf LIST] [--lib LIST] [--recover] [--profile HZ]"""
import collections
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
argv = sys.argv[1:]


def opt(name, default):
    if name in argv:
        i = argv.index(name)
        v = argv[i + 1]
        del argv[i:i + 2]
        return v
    return default


pfs = [int(x) for x in opt("--pf", "").split(",") if x != ""] or [None]
libs = opt("--lib", os.path.join(ROOT, "tools", "libbatchload.so")).split(",")
hz = int(opt("--profile", "0"))
recover = "--recover" in argv
if recover:
    argv.remove("--recover")
runs = int(argv[0]) if argv else 3
k, r, L, nb, e = 16, 4, 1200, 200000, 4
loaded = []
for path in libs:
    lib = C.CDLL(path if os.path.isabs(path) else os.path.join(ROOT, path))
    lib.bl_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.c_uint, C.c_uint, C.c_int,
                           C.c_double, C.c_int, C.POINTER(C.c_double)]
    lib.bl_run_recover.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.c_uint,
                                   C.c_uint, C.c_int, C.c_int, C.POINTER(C.c_double)]
    lib.bl_last_phases.argtypes = [C.POINTER(C.c_double)]
    lib.bl_set_options.argtypes = [C.c_uint, C.c_int, C.c_int, C.c_long]
    lib.bl_set_inflight.argtypes = [C.c_int]
    lib.bl_set_options(0, 0, 1, 32768)  # detail: time every submission
    lib.bl_set_inflight(3)
    lib.bl_set_sampling.argtypes = [C.c_int, C.c_long]
    lib.bl_samples.argtypes = [C.POINTER(C.c_uint64), C.c_long]
    lib.bl_samples.restype = C.c_long
    loaded.append((os.path.basename(path), lib))


class DlInfo(C.Structure):
    _fields_ = [("fname", C.c_char_p), ("fbase", C.c_void_p), ("sname", C.c_char_p), ("saddr", C.c_void_p)]


libdl = C.CDLL(None)
libdl.dladdr.argtypes = [C.c_void_p, C.POINTER(DlInfo)]
samples = collections.defaultdict(collections.Counter)


def resolve(pcs):
    """{pc: (function, file:line)} through dladdr (object and base) and addr2line (static functions too)"""
    by_obj = collections.defaultdict(list)
    out = {}
    for pc in pcs:
        info = DlInfo()
        if not libdl.dladdr(C.c_void_p(pc), C.byref(info)) or not info.fname:
            out[pc] = ("?", "?")
            continue
        by_obj[(info.fname.decode(), info.fbase or 0)].append(pc)
    for (obj, base), lst in by_obj.items():
        offs = [hex(pc - base) for pc in lst]
        try:
            r = subprocess.run(["addr2line", "-f", "-C", "-e", obj] + offs, capture_output=True, text=True, timeout=120)
            lines = r.stdout.splitlines()
        except (OSError, subprocess.SubprocessError):
            lines = []
        name = os.path.basename(obj)
        for i, pc in enumerate(lst):
            fn = lines[2 * i] if 2 * i + 1 < len(lines) else "?"
            fl = lines[2 * i + 1] if 2 * i + 1 < len(lines) else "?"
            out[pc] = (f"{fn} [{name}]", os.path.basename(fl.split(" ")[0]))
    return out


modes = ((3, "in place"),) if recover else ((3, "per-connection arenas, rows in place"),
                                            (2, "per-connection arenas, rows staged"))
res = {}
for reg, what in modes:
    for _ in range(runs):
        for name, lib in loaded:
            for pf in pfs:
                if pf is not None:
                    os.environ["PQUIC_FEC_BATCH_PREFETCH"] = str(pf)
                out, ph = (C.c_double * 8)(), (C.c_double * 6)()
                if hz:
                    lib.bl_set_sampling(hz, 4000000)
                if recover:
                    rc = lib.bl_run_recover(0, k, r, L, e, 64, nb, 2048, 2000, 2, reg, out)
                else:
                    rc = lib.bl_run(0, k, r, L, 64, nb, 2048, 2000, 2, 0.0, reg, out)
                lib.bl_last_phases(ph)
                eng, stg, comp, wall, wait, sub = ph
                tag = f"{'recover' if recover else what} | {name} pf {pf}"
                if hz:
                    buf = (C.c_uint64 * 4000000)()
                    n = lib.bl_samples(buf, 4000000)
                    samples[tag].update(buf[:n])
                    lib.bl_set_sampling(0, 0)
                res.setdefault(tag, []).append(out[0])
                # slot waits include the completions polled while waiting, so the harness's own share is at
                # least wall - submit - completions - waits and at most wall - submit - completions
                print(f"{tag}: rc {rc} {out[0]:6.2f} GiB/s p99 {out[2]:6.0f} us | per block: wall "
                      f"{wall * 1e3 / nb:5.0f} ns, submit {sub * 1e3 / nb:5.0f}, completions {comp * 1e3 / nb:5.0f}, "
                      f"slot waits {wait * 1e3 / nb:5.0f} | engine threads busy {eng / wall:4.2f}, stagers "
                      f"{stg / wall:4.2f}", flush=True)
for tag, v in res.items():
    v = sorted(v)
    print(f"median {tag}: {v[len(v) // 2]:6.2f} GiB/s over {len(v)} runs {['%.2f' % x for x in v]}")
for tag, cnt in samples.items():
    tot = sum(cnt.values())
    where = resolve(list(cnt))
    fn, ln = collections.Counter(), collections.Counter()
    for pc, c in cnt.items():
        fn[where[pc][0]] += c
        ln[where[pc][0].split(" ")[0] + " " + where[pc][1]] += c
    print(f"\nprofile {tag}: {tot} samples")
    for f, c in fn.most_common(25):
        print(f"  {100.0 * c / tot:5.1f}%  {f}")
    print("  top lines:")
    for f, c in ln.most_common(30):
        print(f"  {100.0 * c / tot:5.1f}%  {f}")
