"""Where the batching adapter's latency tail at 512 connections comes from (verdict round 5, weak 7): saturated
generate through pquic_fec_batch_generate (tools/batch_load.c bl_run, one 16 MiB registered arena per
connection, rows in place), 64 against 512 connections, arenas on 4 KiB or transparent huge pages, batch size
and batches in flight; several runs each, the latency quantiles of every run (p50 / p90 / p99 / p99.9 / max).
Runs without torch, as bench.py's host legs do.
usage: python tools/conn512_probe.py [runs] [nconn:batch:inflight:hugepages ...]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "tools", "libbatchload.so"))
D = C.POINTER(C.c_double)
lib.bl_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.c_uint, C.c_uint, C.c_int, C.c_double,
                       C.c_int, D]
lib.bl_set_inflight.argtypes = [C.c_int]
lib.bl_set_options.argtypes = [C.c_uint, C.c_int, C.c_int, C.c_long]
lib.bl_last_latency.argtypes = [D]
lib.bl_last_phases.argtypes = [D]
lib.bl_last_jobs.argtypes = [D]
REG, PER_CONN = 1, 2
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
print(f"stagers {os.environ.get('PQUIC_FEC_BATCH_STAGERS', 'default')}, cpu quota "
      f"{open('/sys/fs/cgroup/cpu.max').read().strip() if os.path.exists('/sys/fs/cgroup/cpu.max') else '?'}",
      flush=True)
sets = [tuple(int(x) for x in a.split(":")) for a in sys.argv[2:]] or \
    [(64, 2048, 3, 0), (512, 2048, 3, 0), (512, 2048, 3, 1), (512, 1024, 3, 0), (512, 2048, 4, 0)]


def cpu_stat():
    """the cgroup's CPU throttling counters (cgroup v2 cpu.stat), or {} where absent"""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {a: int(b) for a, b in (ln.split() for ln in f if ln.strip())}
    except OSError:
        return {}


warm = (C.c_double * 8)()
lib.bl_run(0, 16, 4, 1200, 64, 20000, 2048, 2000, 2, 0.0, REG | PER_CONN, warm)
rc = 0
for nconn, batch, infl, huge in sets:
    lib.bl_set_inflight(infl)
    lib.bl_set_options(0, huge, 0, 0)
    for i in range(runs):
        out, q, ph = (C.c_double * 8)(), (C.c_double * 8)(), (C.c_double * 6)()
        c0 = cpu_stat()
        rc |= lib.bl_run(0, 16, 4, 1200, nconn, 200000, batch, 2000, 2, 0.0, REG | PER_CONN, out)
        c1 = cpu_stat()
        thr = (f"; cgroup throttled {c1.get('nr_throttled', 0) - c0.get('nr_throttled', 0)} times, "
               f"{(c1.get('throttled_usec', 0) - c0.get('throttled_usec', 0)) / 1e3:.1f} ms") if c0 else ""
        lib.bl_last_latency(q)
        lib.bl_last_phases(ph)
        jb = (C.c_double * 3)()
        lib.bl_last_jobs(jb)
        print(f"{nconn:3d} conn batch {batch} inflight {infl} hugepages {huge} run {i}: {out[0]:6.2f} GiB/s, "
              f"latency us p50 {q[0]:6.0f} p90 {q[1]:6.0f} p95 {q[2]:6.0f} p99 {q[3]:6.0f} p99.9 {q[4]:6.0f} "
              f"max {q[5]:6.0f} mean {q[6]:6.0f}; batches {out[4]:.0f}; sender waits {ph[4] / 1e3:.1f} ms of "
              f"{ph[3] / 1e3:.1f}, engine busy {ph[0] / max(ph[3], 1):.2f}; jobs allocated {jb[0]:.0f} "
              f"({jb[1] / 1e3:.1f} ms){thr}", flush=True)
lib.bl_set_options(0, 0, 0, 0)
sys.exit(1 if rc else 0)
