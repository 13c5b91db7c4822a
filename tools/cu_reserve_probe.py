"""The synchronous hooks beside a PCIe-saturating bulk job (tools/batch_load.c bl_hook_latency_loaded: 2000
generate and 2000 recover hooks beside back-to-back 4096-block zero-copy encodes) under two ways of keeping
the hooks fast: slicing the bulk calls (host_path.hip Pacer, knob yield_slice_kb) and reserving CUs for the
block service's worker (knob svc_reserve_cus: the worker's stream on the last n CUs, the host-path streams on
the others).  Each setting runs in a fresh process without torch (as bench.py's host legs do), since the
streams take their CU masks when the service and the contexts are created.
A third field sets knob host_alloc (0 the runtime's default page-locked memory, 1 fine-grained, 2
coarse-grained) for every fecgpu_host_alloc of the process: the bulk job's rows and the hooks' buffers.
A fourth sets knob zc_cus (the host-path streams on that many CUs spread over the chip: fewer waves of the
bulk job reading host memory at once).
usage: python tools/cu_reserve_probe.py [ncalls] [reserve:slice_kb[:host_alloc[:zc_cus]] ...]"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(ncalls, reserve, slice_kb, host_alloc=0, zc_cus=0):
    lib = C.CDLL(os.path.join(ROOT, "pquic_amd", "lib", "libpquic_fec.so"))
    lib.fecgpu_set_knob.argtypes = [C.c_char_p, C.c_int]
    assert lib.fecgpu_set_knob(b"svc_reserve_cus", reserve) == 0
    assert lib.fecgpu_set_knob(b"yield_slice_kb", slice_kb) == 0
    assert lib.fecgpu_set_knob(b"host_alloc", host_alloc) == 0
    assert lib.fecgpu_set_knob(b"zc_cus", zc_cus) == 0
    bl = C.CDLL(os.path.join(ROOT, "tools", "libbatchload.so"))
    D = C.POINTER(C.c_double)
    bl.bl_bulk_rate.argtypes = [C.c_int, C.c_int, C.c_int, D]
    out = (C.c_double * 2)()
    rc = bl.bl_bulk_rate(0, 4096, 200, out)
    bulk_alone = out[0]
    bl.bl_hook_latency_loaded.argtypes = [C.c_int, C.c_int, C.c_long, D]
    lo = (C.c_double * 11)()
    rc |= bl.bl_hook_latency_loaded(0, 4096, ncalls, lo)
    bl.bl_hook_latency.argtypes = [C.c_int] * 5 + [C.c_long, D]
    idle = (C.c_double * 7)()
    rc |= bl.bl_hook_latency(0, 16, 4, 1200, 4, ncalls, idle)
    print(f"reserve {reserve} CUs, slices {slice_kb:5d} KiB, host_alloc {host_alloc}, zc_cus {zc_cus}: rc {rc}; idle hooks generate p50 {idle[0]:.0f} p99 "
          f"{idle[1]:.0f} us, recover p50 {idle[3]:.0f} p99 {idle[4]:.0f} us; loaded generate p50 {lo[0]:.0f} p99 "
          f"{lo[1]:.0f} us, recover p50 {lo[3]:.0f} p99 {lo[4]:.0f} us, withdrawn {lo[8]:.0f}; bulk alone "
          f"{bulk_alone:.3f} ms per call, beside the hooks {lo[9]:.3f} ms (x{lo[9] / bulk_alone:.3f}) over "
          f"{lo[7]:.0f} calls, max {lo[10]:.2f} ms", flush=True)
    return rc


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        sys.exit(1 if child(*(int(x) for x in sys.argv[2:])) else 0)
    ncalls = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    sets = [(tuple(int(x) for x in a.split(":")) + (0, 0, 0))[:5] for a in sys.argv[2:]] or \
        [(0, 2304, 0, 0, 0), (0, 0, 0, 0, 0), (1, 0, 0, 0, 0)]
    rc = 0
    for reserve, kb, ha, zc, _ in sets:
        p = subprocess.run([sys.executable, __file__, "--child", str(ncalls), str(reserve), str(kb), str(ha), str(zc)],
                           timeout=300)
        rc |= p.returncode
        if p.returncode:
            break
    sys.exit(rc)
