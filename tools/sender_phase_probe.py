"""Where one sender thread's time goes at the saturated generate rate (tools/batch_load.c bl_run with
per-connection arenas, batches of 2048, 3 in flight -- the bench leg's setting): per block, the caller's
nanoseconds inside pquic_fec_batch_generate (submission: the protocol operation's allocations, queueing),
inside completions (poll: attach, done, the harness's frees), waiting for a free slot, and the rest (the
harness building its blocks), next to the batcher's engine- and stager-thread time.
usage: python tools/sender_phase_probe.py [runs]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "tools", "libbatchload.so"))
lib.bl_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.c_uint, C.c_uint, C.c_int,
                       C.c_double, C.c_int, C.POINTER(C.c_double)]
lib.bl_last_phases.argtypes = [C.POINTER(C.c_double)]
lib.bl_set_options.argtypes = [C.c_uint, C.c_int, C.c_int, C.c_long]
lib.bl_set_inflight.argtypes = [C.c_int]
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
k, r, L, nb = 16, 4, 1200, 200000
lib.bl_set_options(0, 0, 1, 32768)  # detail: time every submission
lib.bl_set_inflight(3)
for reg, what in ((3, "per-connection arenas, rows in place"), (2, "per-connection arenas, rows staged")):
    for _ in range(runs):
        out, ph = (C.c_double * 8)(), (C.c_double * 6)()
        rc = lib.bl_run(0, k, r, L, 64, nb, 2048, 2000, 2, 0.0, reg, out)
        lib.bl_last_phases(ph)
        eng, stg, comp, wall, wait, sub = ph
        # slot waits include the completions polled while waiting, so the harness's own share is at
        # least wall - submit - completions - waits and at most wall - submit - completions
        print(f"{what}: rc {rc} {out[0]:6.2f} GiB/s p99 {out[2]:6.0f} us | per block: wall {wall * 1e3 / nb:5.0f} ns, "
              f"submit {sub * 1e3 / nb:5.0f}, completions {comp * 1e3 / nb:5.0f}, slot waits {wait * 1e3 / nb:5.0f} "
              f"| engine threads busy {eng / wall:4.2f}, stagers {stg / wall:4.2f}", flush=True)
