"""Saturated batching-adapter throughput (tools/batch_load.c bl_run, k16 r4 L1200, 64 connections)
over stager counts (PQUIC_FEC_BATCH_STAGERS), batch sizes and stream counts, rows gathered from the
registered arena (reg 1) or staged by copies (reg 0), to find the pipeline's bound.
usage (GPU box): python tools/batch_sweep.py [stagers,...] [batch,...] [reg,...] [streams,...] [engines,...]
(engines: PQUIC_FEC_BATCH_ENGINES, engine threads each with its own streams)"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "tools", "libbatchload.so"))
lib.bl_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.c_uint, C.c_uint, C.c_int,
                       C.c_double, C.c_int, C.POINTER(C.c_double)]
stagers = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,4,8,12,15").split(",")]
batches = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "4096").split(",")]
regs = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1").split(",")]
streams = [int(x) for x in (sys.argv[4] if len(sys.argv) > 4 else "2").split(",")]
engines = [int(x) for x in (sys.argv[5] if len(sys.argv) > 5 else "2").split(",")]
for ne, ns in ((e, n) for e in engines for n in stagers):
    os.environ["PQUIC_FEC_BATCH_ENGINES"] = str(ne)
    if ns:
        os.environ["PQUIC_FEC_BATCH_STAGERS"] = str(ns)
    else:
        os.environ.pop("PQUIC_FEC_BATCH_STAGERS", None)
    for batch in batches:
        for reg in regs:
            for nst in streams:
                out = (C.c_double * 8)()
                rc = lib.bl_run(0, 16, 4, 1200, 64, 300000, batch, 2000, nst, 0.0, reg, out)
                print(f"engines {ne} stagers {ns or 'default':>7} batch {batch:5d} reg {reg} streams {nst}: rc {rc} {out[0]:6.2f} "
                      f"GiB/s  p50 {out[1]:7.0f} us  p99 {out[2]:7.0f} us  batches {int(out[4])}", flush=True)
