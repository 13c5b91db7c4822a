"""The synchronous hooks under a bulk job, in a process shaped like bench.py's: torch initialised, the
engine's device path used on several streams first (so the HIP runtime has spread its streams over
its hardware queues), then tools/batch_load.c bl_hook_latency_loaded.  Prints the hook percentiles and
how many bulk calls ran meanwhile and how long the longest took -- a resident block-service worker that
shares a hardware queue with the bulk job holds every bulk kernel behind it.
usage: [LD_LIBRARY_PATH=dir] python tools/hook_load_probe.py [dir/libpquic_fec.so]
(another build: set LD_LIBRARY_PATH to its directory too, so libbatchload.so binds the same file)"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pquic_amd import Engine  # noqa: E402

eng = Engine(0, sys.argv[1]) if len(sys.argv) > 1 else Engine(0)
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
lib.bl_hook_latency.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, D]
lib.bl_hook_latency_loaded.argtypes = [C.c_int, C.c_int, C.c_long, D]
for rep_ in range(2):
    out = (C.c_double * 7)()
    rc = lib.bl_hook_latency(0, 16, 4, 1200, 4, 2000, out)
    print(f"idle:   rc {rc} generate p50 {out[0]:.0f} p99 {out[1]:.0f} us, recover p50 {out[3]:.0f} p99 {out[4]:.0f} us",
          flush=True)
    lo = (C.c_double * 11)()
    rc = lib.bl_hook_latency_loaded(0, 4096, 2000, lo)
    print(f"loaded: rc {rc} generate p50 {lo[0]:.0f} p99 {lo[1]:.0f} us, recover p50 {lo[3]:.0f} p99 {lo[4]:.0f} us; "
          f"bulk calls meanwhile {lo[7]:.0f} (mean {lo[9]:.2f} ms, max {lo[10]:.2f} ms), withdrawn {lo[8]:.0f}",
          flush=True)

# The same hooks beside a DEVICE-resident bulk job (k16 r4 encodes of 4096 blocks in HBM, back to back,
# from a Python thread on its own stream; ctypes releases the GIL while the hooks run): no PCIe traffic
# competes with the hooks' rows, only the GPU's compute units.
import threading  # noqa: E402
import time  # noqa: E402

bsrc = torch.empty((4096, k, L), dtype=torch.uint8, device=dev)
eng.synth_fill(bsrc, bsrc.numel(), 2, 0)
brep = torch.empty((4096, r, L), dtype=torch.uint8, device=dev)
stop, calls, durs = False, [0], []


def bulk():
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        while not stop:
            t0 = time.perf_counter()
            for _ in range(8):
                eng.rlc_encode(bsrc, brep, k, r, L)
            s.synchronize()
            durs.append((time.perf_counter() - t0) * 1e3 / 8)
            calls[0] += 8


th = threading.Thread(target=bulk)
th.start()
time.sleep(0.5)
for rep_ in range(2):
    out = (C.c_double * 7)()
    c0 = calls[0]
    rc = lib.bl_hook_latency(0, 16, 4, 1200, 4, 2000, out)
    print(f"device bulk: rc {rc} generate p50 {out[0]:.0f} p99 {out[1]:.0f} us, recover p50 {out[3]:.0f} p99 "
          f"{out[4]:.0f} us; bulk encodes meanwhile {calls[0] - c0} ({sum(durs[-20:]) / max(1, len(durs[-20:])):.3f} ms each)",
          flush=True)
stop = True
th.join()
