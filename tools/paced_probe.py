"""The paced batching leg (bench.py batch_paced_2GiBps: one sender, 64 connections, 2 GiB/s offered, 250 us
deadline, 4096-block jobs, k16 r4 L1200, registered per-connection arenas) run again and again in one process,
after the bench's own saturated legs, with its latency quantiles and the jobs the batcher allocated on the
sender's thread (tools/batch_load.c bl_last_latency / bl_last_jobs).  The round-6 final bench line, under a
kernel trace, had this leg at p99 8.2 ms / max 41.9 ms with 2 such allocations, against p99 ~0.3 ms in other
runs: how often, and is the allocation the cause or a consequence?
usage (GPU box): python tools/paced_probe.py [runs] [saturated_first]"""
import ctypes as C
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "tools", "libbatchload.so"))
D = C.POINTER(C.c_double)
lib.bl_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.c_uint, C.c_uint, C.c_int, C.c_double,
                       C.c_int, D]
lib.bl_set_inflight.argtypes = [C.c_int]
lib.bl_last_jobs.argtypes = [D]
lib.bl_last_latency.argtypes = [D]
REG, PER_CONN = 1, 2
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
sat_first = int(sys.argv[2]) if len(sys.argv) > 2 else 1
reserves = sys.argv[3].split(",") if len(sys.argv) > 3 and sys.argv[3] != "-" else [None]
hog_ms = int(sys.argv[4]) if len(sys.argv) > 4 else 0
hog = C.CDLL(os.path.join(ROOT, "tests", "host", "libgpuhog.so")) if hog_ms else None


def stall():
    time.sleep(0.6)
    assert hog.gpu_hog_launch(hog_ms) == 0
    assert hog.gpu_hog_wait() == 0


lib.bl_set_inflight(3)
warm = (C.c_double * 8)()
rc = lib.bl_run(0, 16, 4, 1200, 64, 20000, 2048, 2000, 2, 0.0, REG | PER_CONN, warm)
if sat_first:  # the legs bench.py runs before this one
    for nconn in (64, 512):
        rc |= lib.bl_run(0, 16, 4, 1200, nconn, 200000, 2048, 2000, 2, 0.0, REG | PER_CONN, warm)
    print(f"saturated legs first: rc {rc}", flush=True)
for i in range(runs):
    res = reserves[i % len(reserves)]
    if res is not None:
        small, reserve, hold = (res.split(":") + ["1"])[:3]
        os.environ["PQUIC_FEC_BATCH_SMALL"] = small
        os.environ["PQUIC_FEC_BATCH_RESERVE"] = reserve
        os.environ["PQUIC_FEC_BATCH_HOLD"] = hold
    out, q, jb = (C.c_double * 8)(), (C.c_double * 8)(), (C.c_double * 3)()
    th = threading.Thread(target=stall) if hog else None
    if th:
        th.start()
    rc |= lib.bl_run(0, 16, 4, 1200, 64, 100000, 4096, 250, 2, 2.0, REG | PER_CONN, out)
    if th:
        th.join()
    lib.bl_last_latency(q)
    lib.bl_last_jobs(jb)
    print(f"run {i}{'' if res is None else ' small:reserve:hold ' + res}: {out[0]:5.2f} GiB/s, {out[4]:5.0f} batches of {out[7]:5.1f} blocks; latency p50 {q[0]:6.0f} p90 "
          f"{q[1]:6.0f} p99 {q[3]:6.0f} p99.9 {q[4]:6.0f} max {q[5]:6.0f} us; jobs allocated on the sender "
          f"{jb[0]:.0f} ({jb[1] / 1e3:.1f} ms), polls holding for a job {jb[2]:.0f}", flush=True)
sys.exit(1 if rc else 0)
