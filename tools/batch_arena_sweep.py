"""Batching adapter with one registered 16 MiB arena per connection (PQUIC's topology: every connection
owns its plugin instances and their memory, picoquic_internal.h:523,576, plugin.c:835,946-950):
saturated generate at 64 / 512 connections over batch sizes and batches in flight, the receive side
(bl_run_recover), and the synchronous hooks while a bulk job runs (bl_hook_latency_loaded).
    python tools/batch_arena_sweep.py [quick]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "tools", "libbatchload.so"))
D = C.POINTER(C.c_double)
lib.bl_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.c_uint, C.c_uint, C.c_int, C.c_double,
                       C.c_int, D]
lib.bl_run_recover.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.c_uint, C.c_uint,
                               C.c_int, C.c_int, D]
lib.bl_set_inflight.argtypes = [C.c_int]
lib.bl_last_rows.argtypes = [D]
lib.bl_hook_latency_loaded.argtypes = [C.c_int, C.c_int, C.c_long, D]
quick = "quick" in sys.argv


def line(tag, out, rows=None):
    extra = f" rows in place {rows[0]:.0f} staged {rows[1]:.0f}" if rows else ""
    print(f"{tag:52s} {out[0]:6.2f} GiB/s p50 {out[1]:6.0f} p99 {out[2]:6.0f} max {out[3]:6.0f} us "
          f"batches {out[4]:5.0f}{extra}", flush=True)


for nconn in (64, 512):
    for batch, infl in ((4096, 4), (4096, 2), (2048, 4), (2048, 3)) if not quick else ((4096, 2),):
        lib.bl_set_inflight(infl)
        for reg, name in ((3, "per-connection arenas, registered"), (1, "one arena, registered")):
            if reg == 1 and nconn == 512:
                continue
            out, rows = (C.c_double * 8)(), (C.c_double * 2)()
            rc = lib.bl_run(0, 16, 4, 1200, nconn, 200000, batch, 2000, 2, 0.0, reg, out)
            lib.bl_last_rows(rows)
            line(f"gen {nconn:3d} conn batch {batch} inflight {infl} {name}" if not rc else f"rc {rc}", out, rows)
lib.bl_set_inflight(2)
for nconn in (64, 512):
    for reg in (3, 2):
        out, rows = (C.c_double * 8)(), (C.c_double * 2)()
        rc = lib.bl_run_recover(0, 16, 4, 1200, 4, nconn, 200000, 4096, 2000, 2, reg, out)
        lib.bl_last_rows(rows)
        line(f"rec {nconn:3d} conn e4 batch 4096 {'registered' if reg & 1 else 'staged'} rc {rc}", out, rows)
        print(f"    recovered symbols {out[6]:.0f}", flush=True)
for bulk in (0, 4096):
    out = (C.c_double * 11)()
    if bulk:
        rc = lib.bl_hook_latency_loaded(0, bulk, 2000, out)
    else:
        lib.bl_hook_latency.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, D]
        rc = lib.bl_hook_latency(0, 16, 4, 1200, 4, 2000, out)
    print(f"hooks, bulk {bulk:4d} blocks: rc {rc} generate p50 {out[0]:.0f} p99 {out[1]:.0f} us, recover p50 "
          f"{out[3]:.0f} p99 {out[4]:.0f} us, bulk calls {out[7]:.0f} (mean {out[9]:.2f} max {out[10]:.2f} ms), "
          f"withdrawn {out[8]:.0f}", flush=True)
