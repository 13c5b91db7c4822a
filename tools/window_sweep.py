"""Sliding-window sender through the batching adapter (tools/batch_load.c bl_run_window): windows of
the last k symbols every `step` new ones, 64 connections, L 1200, through pquic_fec_batch_generate_window
(api 1: shared streams + the shared-coefficient kernel) and pquic_fec_batch_generate (api 0: every
window a block).  The redundancy controllers set the shapes: constant (N 6, K 5: a repair every 5
symbols over the <= 30 in flight, window_framework_sender.h:7, constant_redundancy_controller.h:1-2)
and N 30 / K 25 (uniform / burst controllers).
usage (GPU box): python tools/window_sweep.py [k:r:step,...] [batch] [windows]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "tools", "libbatchload.so"))
lib.bl_run_window.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.c_uint, C.c_uint,
                              C.c_int, C.c_int, C.POINTER(C.c_double)]
shapes = [tuple(int(v) for v in x.split(":")) for x in (sys.argv[1] if len(sys.argv) > 1 else
                                                          "30:1:5,30:5:25,30:4:10,32:8:8,30:4:1").split(",")]
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
nwin = int(sys.argv[3]) if len(sys.argv) > 3 else 200000
for k, r, step in shapes:
    for api in (1, 0):
        out = (C.c_double * 8)()
        rc = lib.bl_run_window(0, k, r, 1200, step, 64, nwin, batch, 2000, 2, api, out)
        print(f"k{k:2d} r{r} step {step:2d} api {'window' if api else 'block '}: rc {rc} stream {out[0]:6.2f} GiB/s "
              f"(windows {out[7]:7.2f} GiB/s)  p50 {out[1]:7.0f} us  p99 {out[2]:7.0f} us  batches {int(out[4])}",
              flush=True)
