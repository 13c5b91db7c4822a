"""Senders (tools/batch_load.c bl_run_senders: sender threads, each with its own batcher and 64
connections, per-connection registered arenas, k16 r4 L1200) over batches in flight, batch size and the
batcher's flush delay: which settings keep the aggregate rate at or above 40 GiB/s with p99 <= 5 ms.
No torch in this process (the bench runs its host legs the same way).
usage (GPU box): python tools/senders_sweep.py [inflight,...] [batch,...] [delay_us,...] [runs] [senders]"""
import ctypes as C
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "tools", "libbatchload.so"))
D = C.POINTER(C.c_double)
lib.bl_run_senders.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.c_uint, C.c_uint,
                               C.c_int, C.c_int, D]
lib.bl_set_inflight.argtypes = [C.c_int]
inflights = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,3").split(",")]
batches = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1024,1536,2048").split(",")]
delays = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "2000").split(",")]
runs = int(sys.argv[4]) if len(sys.argv) > 4 else 3
nsend = int(sys.argv[5]) if len(sys.argv) > 5 else 2
REG, PER_CONN = 1, 2
# configurations alternate within each round, so a drift of the box's CPU share spreads over all of them
configs = [(i, b, d) for i in inflights for b in batches for d in delays]
res = {c: [] for c in configs}
for rnd in range(runs):
    for inflight, batch, delay in configs:
        lib.bl_set_inflight(inflight)
        out = (C.c_double * 8)()
        rc = lib.bl_run_senders(nsend, 0, 16, 4, 1200, 64, 200000, batch, delay, 2, REG | PER_CONN, out)
        if rc:
            print(f"inflight {inflight} batch {batch} delay {delay}: rc {rc}", flush=True)
            sys.exit(1)
        res[(inflight, batch, delay)].append(list(out))
        print(f"  round {rnd} inflight {inflight} batch {batch} delay {delay}: {out[0]:.2f} GiB/s p99 {out[2]:.0f} us",
              flush=True)
for (inflight, batch, delay), rs in res.items():
    med = sorted(rs, key=lambda o: o[0])[len(rs) // 2]
    print(f"senders {nsend} inflight {inflight} batch {batch:5d} delay {delay:5d}: median {med[0]:6.2f} GiB/s p50 "
          f"{med[1]:6.0f} p99 {med[2]:6.0f} us | runs " + " ".join(f"{o[0]:.1f}/{o[2]:.0f}" for o in rs) +
          f" | p99 median {statistics.median(o[2] for o in rs):.0f}", flush=True)
