"""Where the batching adapter's saturated generate rate goes (tools/batch_load.c).

1. bl_rows_probe: the gathered engine call alone (fecgpu_rlc_encode_rows_host on rows in a registered
   arena) against the same blocks in contiguous page-locked rows (fecgpu_rlc_encode_host, zero-copy);
2. bl_run saturated (the bench leg's configuration) with the batcher's thread times: engine-thread,
   stager-thread and caller-completion microseconds against the wall clock.
Usage: python tools/rows_probe.py [runs]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "tools", "libbatchload.so"))
lib.bl_rows_probe.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.c_int, C.c_int, C.POINTER(C.c_double)]
lib.bl_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.c_uint, C.c_uint, C.c_int,
                       C.c_double, C.c_int, C.POINTER(C.c_double)]
lib.bl_last_phases.argtypes = [C.POINTER(C.c_double)]
lib.bl_set_options.argtypes = [C.c_uint, C.c_int, C.c_int, C.c_long]
lib.bl_clock_cost.restype = C.c_double
lib.bl_run_senders.argtypes = [C.c_int] + lib.bl_run.argtypes[:9] + [C.c_int, C.POINTER(C.c_double)]
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
k, r, L = 16, 4, 1200
for nb in (4096,):
    for mode in (1,):
        out = (C.c_double * 4)()
        rc = lib.bl_rows_probe(0, k, r, L, nb, 20, mode, out)
        print(f"rows_probe blocks {nb:5d} mode {mode} ({'64-block source pool' if mode == 0 else 'distinct sources'}): "
              f"rc {rc}  gathered {out[0]:6.2f} GiB/s {out[1]:6.3f} ms/call   contiguous page-locked {out[2]:6.2f} GiB/s "
              f"{out[3]:6.3f} ms/call", flush=True)
print(f"now_us(): {lib.bl_clock_cost():.1f} ns per call", flush=True)
lib.bl_set_options(0, 0, 0, 32768)
for _ in range(runs):
    out = (C.c_double * 8)()
    rc = lib.bl_run(0, k, r, L, 64, 200000, 4096, 2000, 2, 0.0, 1, out)
    print(f"bl_run (caller thread)  : rc {rc} {out[0]:6.2f} GiB/s p50 {out[1]:6.0f} p99 {out[2]:6.0f} max {out[3]:6.0f} us "
          f"batches {int(out[4])} wall {out[5]:.3f} s", flush=True)
    for ns in (1, 2):
        out = (C.c_double * 8)()
        rc = lib.bl_run_senders(ns, 0, k, r, L, 64, 200000, 4096, 2000, 2, 1, out)
        print(f"bl_run_senders {ns}       : rc {rc} {out[0]:6.2f} GiB/s p50 {out[1]:6.0f} p99 {out[2]:6.0f} max {out[3]:6.0f} us "
              f"batches {int(out[4])} wall {out[5]:.3f} s", flush=True)
