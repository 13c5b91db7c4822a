"""Where a slow hook's time goes while a PCIe-saturating bulk job runs (verdict round 5, weak 6).  A bulk
thread runs back-to-back zero-copy fecgpu_rlc_encode_host calls (4096 k16 r4 blocks in page-locked memory,
unsliced: knob yield_slice_kb 0) while this thread makes single-block calls through the resident block
service; after each call fecgpu_block_svc_last_stamps gives the worker's clock at claim / request in LDS / rows
coded / before `done`, and the host's post and done-seen times.  The device clock is mapped onto the host's
with the median offset of the fast calls, so each slow call splits into: posted -> claimed (the worker had
not seen it), claimed -> coded (reading the request and the rows over PCIe, computing, writing), coded ->
done published (the release fence), published -> seen by the host.
usage (GPU box): python tools/svc_phase_probe.py [calls] [slice_kb] [svc_reserve_cus]"""
import ctypes as C
import os
import statistics
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from pquic_amd import load_library  # noqa: E402

ncalls = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
slice_kb = int(sys.argv[2]) if len(sys.argv) > 2 else 0
reserve = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # knob svc_reserve_cus (before the streams exist)
lib = load_library()
lib.fecgpu_set_knob.argtypes = [C.c_char_p, C.c_int]
assert lib.fecgpu_set_knob(b"yield_slice_kb", slice_kb) == 0
assert lib.fecgpu_set_knob(b"svc_reserve_cus", reserve) == 0
print(f"slices {slice_kb} KiB, svc_reserve_cus {reserve}", flush=True)
lib.fecgpu_host_alloc.restype = C.c_void_p
lib.fecgpu_host_alloc.argtypes = [C.c_size_t]
lib.fecgpu_host_ctx_create.restype = C.c_void_p
lib.fecgpu_host_ctx_create.argtypes = [C.c_int, C.c_int, C.c_size_t]
k, r, L, nb = 16, 4, 1200, 4096
src = lib.fecgpu_host_alloc(nb * k * L)
rep = lib.fecgpu_host_alloc(nb * r * L)
C.memset(src, 0x5A, nb * k * L)
ctx = lib.fecgpu_host_ctx_create(0, 4, 64 << 20)
svc = lib.fecgpu_block_svc_create(0)
assert src and rep and ctx and svc
assert lib.fecgpu_block_svc_set_deadline(svc, 1_000_000) == 0
hs = lib.fecgpu_host_alloc(k * L)
hr = lib.fecgpu_host_alloc(r * L)
C.memset(hs, 0x33, k * L)

stop = threading.Event()
bulk_calls = [0]


def bulk():
    while not stop.is_set():
        assert lib.fecgpu_rlc_encode_host(ctx, src, rep, nb, k, r, L, 0, None) == 0
        bulk_calls[0] += 1


rows = []
st = (C.c_uint64 * 6)()
for phase in ("idle", "loaded"):
    th = None
    if phase == "loaded":
        th = threading.Thread(target=bulk, daemon=True)
        th.start()
        while bulk_calls[0] < 2:
            pass
    res = []
    for i in range(ncalls):
        assert lib.fecgpu_block_svc_rlc_encode(svc, hs, hr, k, r, L, i & 0xFFFFFF) == 0
        assert lib.fecgpu_block_svc_last_stamps(svc, st) == 0
        res.append(tuple(st))
    if th:
        stop.set()
        th.join()
    tot = [s[5] - s[4] for s in res]
    fast = [s for s in res if s[5] - s[4] <= sorted(tot)[len(tot) // 4]]
    # device ticks (10 ns) -> host us: offset = median over fast calls of (claim tick / 100 - post us)
    off = statistics.median(s[0] / 100.0 - s[4] for s in fast)

    def split(s):
        claim = s[0] / 100.0 - off
        return (claim - s[4], (s[2] - s[0]) / 100.0, (s[3] - s[2]) / 100.0, s[5] - (s[3] / 100.0 - off))

    parts = [split(s) for s in res]
    srt = sorted(range(len(res)), key=lambda j: tot[j])
    print(f"{phase}: {ncalls} calls, p50 {tot[srt[len(srt) // 2]]} us, p90 {tot[srt[int(len(srt) * .9)]]} us, "
          f"p99 {tot[srt[int(len(srt) * .99)]]} us, max {tot[srt[-1]]} us; bulk calls {bulk_calls[0]}", flush=True)
    for name, sel in (("fastest half", srt[:len(srt) // 2]), ("slowest 5 %", srt[-max(1, len(srt) // 20):])):
        med = [statistics.median(parts[j][c] for j in sel) for c in range(4)]
        print(f"  {name:13s} medians (us): posted->claimed {med[0]:8.1f}  claimed->coded {med[1]:8.1f}  "
              f"coded->done published {med[2]:7.1f}  published->seen {med[3]:8.1f}", flush=True)
    for j in srt[-5:]:
        p = parts[j]
        print(f"    slow call {j}: total {tot[j]} us = posted->claimed {p[0]:.1f}, claimed->coded {p[1]:.1f}, "
              f"coded->published {p[2]:.1f}, published->seen {p[3]:.1f}", flush=True)
lib.fecgpu_block_svc_destroy(svc)
