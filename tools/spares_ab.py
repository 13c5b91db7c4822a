"""Spare jobs (the batcher's provisioner thread, batch.c prov_main) on and off, alternating run by run in one
process (PQUIC_FEC_BATCH_SPARES is read per batcher): one sender at 64 and 512 connections and two senders
(tools/batch_load.c bl_run / bl_run_senders, registered per-connection arenas, k16 r4 L1200), rate and latency.
usage (GPU box): python tools/spares_ab.py [runs]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "tools", "libbatchload.so"))
D = C.POINTER(C.c_double)
lib.bl_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.c_uint, C.c_uint, C.c_int, C.c_double,
                       C.c_int, D]
lib.bl_run_senders.argtypes = [C.c_int] + lib.bl_run.argtypes[:9] + [C.c_int, D]
lib.bl_set_inflight.argtypes = [C.c_int]
lib.bl_last_jobs.argtypes = [D]
REG, PER_CONN = 1, 2
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
lib.bl_set_inflight(3)
warm = (C.c_double * 8)()
lib.bl_run(0, 16, 4, 1200, 64, 20000, 2048, 2000, 2, 0.0, REG | PER_CONN, warm)
rc = 0
for i in range(runs):
    for spares in ("1", "0"):
        os.environ["PQUIC_FEC_BATCH_SPARES"] = spares
        for name, fn in (("1 sender 64 conn  ", lambda o: lib.bl_run(0, 16, 4, 1200, 64, 200000, 2048, 2000, 2, 0.0,
                                                                  REG | PER_CONN, o)),
                         ("1 sender 512 conn ", lambda o: lib.bl_run(0, 16, 4, 1200, 512, 200000, 2048, 2000, 2, 0.0,
                                                                  REG | PER_CONN, o)),
                         ("2 senders 64 conn ", lambda o: lib.bl_run_senders(2, 0, 16, 4, 1200, 64, 200000, 1024, 2000,
                                                                          2, REG | PER_CONN, o))):
            out, jb = (C.c_double * 8)(), (C.c_double * 3)()
            rc |= fn(out)
            lib.bl_last_jobs(jb)
            jobs = f", jobs allocated on the sender {jb[0]:.0f} ({jb[1] / 1e3:.1f} ms)" if "1 sender" in name else ""
            print(f"run {i} spares {spares}: {name} {out[0]:6.2f} GiB/s p50 {out[1]:6.0f} p99 {out[2]:6.0f} max "
                  f"{out[3]:6.0f} us{jobs}", flush=True)
sys.exit(1 if rc else 0)
