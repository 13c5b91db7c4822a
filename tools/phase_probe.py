"""Phases of a one-block launch (the synchronous hooks' shape), from the s_memrealtime stamps of a
diagnostic build (-DFEC_STAMP: python tools/build_variants.py stamp=FEC_STAMP; fec_engine.hip
FEC_STAMP_AT).  Decode k16 e4 / k32 e8 (k_rlc_decode_small): 0 start, 1 masks read, 2 TinyMT rows
done, 3 plan done, 4 data pass + stores done; wide systems (e > 8, the LDS wave plan) 8 sorted, 9
eliminated, 10 back-substituted.  Encode (k_rlc_encode_bs): 5 start, 6 coefficient rows
done, 7 data pass + stores done.  Device-resident buffers and page-locked host buffers (zero copy),
median over many launches, in microseconds; plus the wall time per launch + sync.
usage: python tools/phase_probe.py [lib]"""
import ctypes as C
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pquic_amd import Engine  # noqa: E402

lib_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "pquic_amd/lib/variants/stamp/libpquic_fec.so")
eng = Engine(0, lib_path=lib_path)
eng.lib.fecgpu_debug_stamps.argtypes = [C.POINTER(C.c_uint64)]
dev = torch.device("cuda:0")
N = 400


def stamps():
    out = (C.c_uint64 * 16)()
    assert eng.lib.fecgpu_debug_stamps(out) == 0
    return list(out)


def phases(fn, idx):
    walls, rows = [], []
    for it in range(N + 50):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        st = stamps()
        if it >= 50:
            walls.append((t1 - t0) * 1e6)
            rows.append([(st[b] - st[a]) / 100.0 for a, b in zip(idx[:-1], idx[1:])])
    med = [statistics.median(c) for c in zip(*rows)]
    return statistics.median(walls), med


def run(where, k, r, e, L):
    pin = where == "pinned"
    mk = (lambda shape, dt: torch.empty(shape, dtype=dt).pin_memory()) if pin else \
        (lambda shape, dt: torch.empty(shape, dtype=dt, device=dev))
    src, rep = mk((1, k, L), torch.uint8), mk((1, r, L), torch.uint8)
    tmp = torch.empty((1, k, L), dtype=torch.uint8, device=dev)
    eng.synth_fill(tmp, tmp.numel(), 5, 0)
    src.copy_(tmp)
    sp, rp = mk((1, 2), torch.int64), mk((1, 2), torch.int64)
    s0 = ((1 << k) - 1) & ~((1 << e) - 1)
    sp.copy_(torch.tensor([[s0 - (1 << 64) if s0 >= 1 << 63 else s0, 0]]))  # as int64 (k = 64)
    rp.copy_(torch.tensor([[(1 << r) - 1, 0]]))
    st, rec = mk(1, torch.uint8), mk((1, 2), torch.int64)
    ws = eng.alloc_workspace(1, k, r)
    w_enc, p_enc = phases(lambda: eng.rlc_encode(src, rep, k, r, L), [5, 6, 7])
    # e > 8: the plan is its own kernel (plan_wave_block), stamping 1 (masks), 2 (TinyMT rows), 8 (sorted),
    # 9 (eliminated), 10 (back-substituted); stamps 0, 3, 4 of k_rlc_decode_small do not apply
    wide = (k < r and k or r) > 8
    idx = [1, 2, 8, 9, 10] if wide else [0, 1, 2, 3, 4]
    w_dec, p_dec = phases(lambda: eng.rlc_decode(src, rep, sp, rp, st, rec, k, r, L, workspace=ws), idx)
    print(f"{where:8s} k{k} r{r} e{e}: encode wall {w_enc:6.1f} us | coef rows {p_enc[0]:5.2f} data+store {p_enc[1]:5.2f}")
    if wide:
        print(f"{where:8s} k{k} r{r} e{e}: decode wall {w_dec:6.1f} us | plan: tinymt {p_dec[0]:5.2f} sort {p_dec[1]:5.2f} "
              f"eliminate {p_dec[2]:5.2f} back-substitute {p_dec[3]:5.2f}")
    else:
        print(f"{where:8s} k{k} r{r} e{e}: decode wall {w_dec:6.1f} us | masks {p_dec[0]:5.2f} tinymt {p_dec[1]:5.2f} "
              f"plan {p_dec[2]:5.2f} data+store {p_dec[3]:5.2f}")


for where in ("device", "pinned"):  # pinned: page-locked host memory, which ROCm maps at the same address
    run(where, 16, 4, 4, 1200)
    run(where, 32, 8, 8, 1200)
    run(where, 64, 16, 16, 9000)
