"""One loaded hook-latency run (tools/batch_load.c bl_hook_latency_loaded: 2000 generate and 2000 recover
hooks beside back-to-back 4096-block zero-copy encodes), in a process shaped like bench.py's, writing
every timed call (op, CLOCK_MONOTONIC start us, duration us) to a CSV.  Run it under
`rocprofv3 --kernel-trace --hip-runtime-trace` and line the slow calls up with the trace
(tools/hook_trace_summary.py): which kernel was running, and whether the block-service worker was
waiting to start.
With --sweep, no CSV: the loaded percentiles for bulk calls of 4096, 1024, 512 and 256 blocks (what
slicing the bulk job would buy the hooks, and what it costs the bulk rate).
With --pacer, no CSV: bulk calls of 4096 blocks under several Pacer settings (knobs yield_slice_kb,
yield_depth, yield_gate_us; host_path.hip), the hooks' percentiles against the bulk call's time.
usage: python tools/hook_trace_probe.py OUT_CSV [ncalls] | --sweep [ncalls] | --pacer [ncalls]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pquic_amd import Engine  # noqa: E402

sweep = sys.argv[1] == "--sweep"
pacer = sys.argv[1] == "--pacer"
out_csv = None if sweep or pacer else sys.argv[1]
ncalls = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
eng = Engine(0)
dev = torch.device("cuda:0")
k, r, L, nb = 16, 4, 1200, 1 << 14
src = torch.empty((nb, k, L), dtype=torch.uint8, device=dev)
eng.synth_fill(src, src.numel(), 1, 0)
rep = torch.empty((nb, r, L), dtype=torch.uint8, device=dev)
streams = [torch.cuda.Stream() for _ in range(6)]
for s in streams:
    with torch.cuda.stream(s):
        eng.rlc_encode(src, rep, k, r, L)
        (src[:64].float() * 2).sum()
torch.cuda.synchronize()
lib = C.CDLL(os.path.join(ROOT, "tools", "libbatchload.so"))
D = C.POINTER(C.c_double)
lib.bl_hook_latency_loaded.argtypes = [C.c_int, C.c_int, C.c_long, D]
lib.bl_hook_calls.argtypes = [C.POINTER(C.c_uint64), C.c_long]
lib.bl_hook_calls.restype = C.c_long
rc = 0
if pacer:
    def knobs(kb, depth, gate, streams, always):
        for n, v in (("yield_slice_kb", kb), ("yield_depth", depth), ("yield_gate_us", gate),
                     ("yield_streams", streams), ("yield_always", always)):
            eng.set_knob(n, v)
    # the bulk job alone, slices forced (what slicing costs without any hook)
    lib.bl_bulk_rate.argtypes = [C.c_int, C.c_int, C.c_int, D]
    for kb, streams, depth in (() if os.environ.get("PACER_SETS") else
                               ((0, 1, 4), (2048, 2, 16), (2560, 2, 16), (3072, 2, 16), (4096, 2, 16))):
        knobs(kb, depth, 0, streams, 1)
        out = (C.c_double * 2)()
        rc |= lib.bl_bulk_rate(0, 4096, 200, out)
        print(f"bulk alone, slices {kb:5d} KiB on {streams} stream(s), depth {depth}: {out[0]:.3f} ms per 4096-block call "
              f"({out[1]:.1f} GiB/s of sources)", flush=True)
    sets = ((0, 4, 0, 1), (2048, 16, 0, 2), (2560, 16, 0, 2), (3072, 16, 0, 2), (2048, 12, 0, 2), (4096, 16, 0, 2),
            (2048, 16, 0, 2), (3072, 16, 0, 2), (0, 4, 0, 1))
    if os.environ.get("PACER_SETS"):  # e.g. "2560:16,2304:16,2560:12" (2 streams, no gate)
        sets = tuple((int(a), int(b), 0, 2) for a, b in (x.split(":") for x in os.environ["PACER_SETS"].split(",")))
    for kb, depth, gate, streams in sets:
        knobs(kb, depth, gate, streams, 0)
        s0 = eng.stats()
        lo = (C.c_double * 11)()
        rc |= lib.bl_hook_latency_loaded(0, 4096, ncalls, lo)
        s1 = eng.stats()
        gibs = 4096 * 16 * 1200 / (lo[9] * 1e-3) / 2**30 if lo[9] else 0
        print(f"hooks + bulk, slices {kb:5d} KiB depth {depth:2d} gate {gate:4d} us streams {streams}: generate p50 "
              f"{lo[0]:.0f} p99 {lo[1]:.0f} us, recover p50 {lo[3]:.0f} p99 {lo[4]:.0f} us; bulk {lo[7]:.0f} calls, "
              f"mean {lo[9]:.3f} ms ({gibs:.1f} GiB/s of sources), max {lo[10]:.2f} ms; slices "
              f"{s1['yield_slices'] - s0['yield_slices']}, held {s1['yield_waits'] - s0['yield_waits']}", flush=True)
    sys.exit(0 if rc == 0 else 1)
for bulk in ((4096, 1024, 512, 256) if sweep else (4096,)):
    lo = (C.c_double * 11)()
    rc |= lib.bl_hook_latency_loaded(0, bulk, ncalls, lo)
    gibs = bulk * 16 * 1200 / (lo[9] * 1e-3) / 2**30 if lo[9] else 0
    print(f"bulk {bulk:5d} blocks: rc {rc} generate p50 {lo[0]:.0f} p99 {lo[1]:.0f} us, recover p50 {lo[3]:.0f} "
          f"p99 {lo[4]:.0f} us; bulk calls meanwhile {lo[7]:.0f} (mean {lo[9]:.3f} ms = {gibs:.1f} GiB/s of sources, "
          f"max {lo[10]:.2f} ms), withdrawn {lo[8]:.0f}", flush=True)
if sweep:
    sys.exit(0 if rc == 0 else 1)
buf = (C.c_uint64 * (3 * 2 * ncalls))()
n = lib.bl_hook_calls(buf, 2 * ncalls)
with open(out_csv, "w") as f:
    f.write("op,start_us,dur_us\n")
    for i in range(n):
        f.write(f"{buf[3 * i]},{buf[3 * i + 1]},{buf[3 * i + 2]}\n")
print(f"{n} calls written to {out_csv}")
sys.exit(0 if rc == 0 else 1)
