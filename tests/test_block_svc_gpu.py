"""The resident single-block service (fecgpu_block_svc_*, include/fecgpu.h), which serves the
synchronous hooks one block per call (block_framework_sender.h:187, fec_protoops.h:246) without a
kernel launch: bytes against the oracle, the worker's idle exit and relaunch, and its refusals."""
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle_py import Oracle, synth_bytes  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    from pquic_amd import load_library
    return load_library()


@pytest.fixture(scope="module")
def svc(lib):
    v = lib.fecgpu_block_svc_create(0)
    assert v
    yield v
    lib.fecgpu_block_svc_destroy(v)


def pinned(a):
    t = torch.from_numpy(np.ascontiguousarray(a)).pin_memory()
    return t, t.numpy()


def _decode_case(oracle, k, r, L, seed, rng):
    src = synth_bytes(k * L, seed).reshape(1, k, L)
    seeds = np.array([(int(rng.integers(0, 1 << 24)) << 8) | i for i in range(r)], np.uint32)
    mul, _ = oracle.gf_tables()
    rep = np.zeros((1, r, L), np.uint8)
    for i in range(r):
        c = oracle.coefs(int(seeds[i]), k)
        for j in range(k):
            rep[0, i] ^= mul[c[j]][src[0, j]]
    e = int(rng.integers(0, min(k, r) + 1))
    miss = rng.choice(k, e, replace=False)
    sp = np.zeros((1, 2), np.uint64)
    rp = np.zeros((1, 2), np.uint64)
    for j in range(k):
        if j not in miss:
            sp[0, j >> 6] |= np.uint64(1 << (j & 63))
    for i in rng.choice(r, int(rng.integers(max(0, e - 1), r + 1)), replace=False):
        rp[0, int(i) >> 6] |= np.uint64(1 << (int(i) & 63))
    work = src.copy()
    work[0, miss] = 0
    return src, rep, seeds, sp, rp, work


@pytest.mark.parametrize("k,r,L", [(16, 4, 1200), (32, 8, 1200), (5, 3, 20), (64, 16, 100), (1, 1, 4), (20, 16, 36)])
def test_svc_encode_decode_vs_oracle(lib, svc, k, r, L):
    o = Oracle()
    rng = np.random.default_rng(k * 31 + r)
    for it in range(6):
        fbn = int(rng.integers(0, 1 << 24))
        src = synth_bytes(k * L, 1000 + it).reshape(1, k, L)
        ts, hs = pinned(src)
        tr, hr = pinned(np.zeros((1, r, L), np.uint8))
        assert lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr.data_ptr(), k, r, L, fbn) == 0
        assert np.array_equal(hr, o.rlc_encode_batch(src, r, fbn))
        src, rep, seeds, sp, rp, work = _decode_case(o, k, r, L, 2000 + it, rng)
        tw, hw = pinned(work)
        trp, _ = pinned(rep)
        tseed, _ = pinned(seeds)
        tsp, _ = pinned(sp.view(np.int64))
        trpm, _ = pinned(rp.view(np.int64))
        tst, hst = pinned(np.full(1, 0xEE, np.uint8))
        trec, hrec = pinned(np.zeros((1, 2), np.int64))
        assert lib.fecgpu_block_svc_rlc_decode_seeded(svc, tw.data_ptr(), trp.data_ptr(), tw.data_ptr(), k, r, L,
                                                      tseed.data_ptr(), tsp.data_ptr(), trpm.data_ptr(),
                                                      tst.data_ptr(), trec.data_ptr()) == 0
        blk = [work[0, j].copy() if (int(sp[0, j >> 6]) >> (j & 63)) & 1 else None for j in range(k)]
        reps = [rep[0, i].copy() if (int(rp[0, i >> 6]) >> (i & 63)) & 1 else None for i in range(r)]
        st, out = o.rlc_decode_block(0, blk, reps, rep_seeds=[int(x) for x in seeds])
        assert hst[0] == st
        got_rec = [j for j in range(k) if (int(hrec.view(np.uint64)[0, j >> 6]) >> (j & 63)) & 1]
        assert sorted(got_rec) == sorted(out.keys())
        for j, row in out.items():
            assert np.array_equal(hw[0, j, :len(row)], row)


def test_svc_idle_exit_and_relaunch(lib, svc):
    """The worker ends after 20 ms without a request; the next call relaunches it and is served."""
    o = Oracle()
    k, r, L = 16, 4, 1200
    src = synth_bytes(k * L, 7).reshape(1, k, L)
    ts, _ = pinned(src)
    tr, hr = pinned(np.zeros((1, r, L), np.uint8))
    want = o.rlc_encode_batch(src, r, 99)
    assert lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr.data_ptr(), k, r, L, 99) == 0
    n0 = lib.fecgpu_block_svc_launches(svc)
    for _ in range(50):  # back to back: one worker serves them all
        hr[:] = 0
        assert lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr.data_ptr(), k, r, L, 99) == 0
        assert np.array_equal(hr, want)
    assert lib.fecgpu_block_svc_launches(svc) == n0
    time.sleep(0.1)
    hr[:] = 0
    assert lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr.data_ptr(), k, r, L, 99) == 0
    assert np.array_equal(hr, want)
    assert lib.fecgpu_block_svc_launches(svc) == n0 + 1


def test_svc_refusals(lib, svc):
    """Pageable buffers and blocks too large for the worker are refused (FECGPU_ERR_INVALID = -1),
    so the caller takes the launch path."""
    k, r, L = 16, 4, 1200
    src = np.zeros((1, k, L), np.uint8)  # pageable
    rep = np.zeros((1, r, L), np.uint8)
    assert lib.fecgpu_block_svc_rlc_encode(svc, src.ctypes.data, rep.ctypes.data, k, r, L, 0) == -1
    ts, _ = pinned(np.zeros((1, 20, 36), np.uint8))  # 20 unknowns possible: more than one pass
    tr, _ = pinned(np.zeros((1, 20, 36), np.uint8))
    tm, _ = pinned(np.zeros((1, 2), np.int64))
    tsd, _ = pinned(np.zeros(20, np.uint32))
    tst, _ = pinned(np.zeros(1, np.uint8))
    assert lib.fecgpu_block_svc_rlc_decode_seeded(svc, ts.data_ptr(), tr.data_ptr(), ts.data_ptr(), 20, 20, 36,
                                                  tsd.data_ptr(), tm.data_ptr(), tm.data_ptr(), tst.data_ptr(),
                                                  tm.data_ptr()) == -1
    big_k, big_L = 100, 2000  # 200 KB of rows
    ts, _ = pinned(np.zeros((1, big_k, big_L), np.uint8))
    tr, _ = pinned(np.zeros((1, 4, big_L), np.uint8))
    assert lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr.data_ptr(), big_k, 4, big_L, 0) == -1


def test_svc_deadline_withdraws_and_backs_off(lib, svc):
    """A request no worker has claimed by the deadline is withdrawn (compare-and-swap on the request
    number; a request a worker claimed first is waited for and succeeds), the call returns
    FECGPU_ERR_INVALID so the caller takes the launch path, and the following calls skip the service
    for a while.  A later request is served normally: no withdrawn request is ever served later."""
    o = Oracle()
    k, r, L = 16, 4, 1200
    src = synth_bytes(k * L, 11).reshape(1, k, L)
    ts, _ = pinned(src)
    tr, hr = pinned(np.zeros((1, r, L), np.uint8))
    want = o.rlc_encode_batch(src, r, 5)
    time.sleep(0.05)  # the worker has idled out: the next call launches one
    m0 = lib.fecgpu_block_svc_deadline_misses(svc)
    assert lib.fecgpu_block_svc_set_deadline(svc, 0) == 0
    outcomes = []
    for _ in range(20):
        hr[:] = 0
        rc = lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr.data_ptr(), k, r, L, 5)
        assert rc in (0, -1)
        if rc == 0:
            assert np.array_equal(hr, want)
        outcomes.append(rc)
    misses = lib.fecgpu_block_svc_deadline_misses(svc) - m0
    assert misses >= 1
    assert outcomes.count(-1) >= 1  # withdrawn, or skipped during the back-off
    assert lib.fecgpu_block_svc_set_deadline(svc, 2000) == 0  # also ends the back-off
    for _ in range(5):
        hr[:] = 0
        assert lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr.data_ptr(), k, r, L, 5) == 0
        assert np.array_equal(hr, want)
    assert lib.fecgpu_block_svc_deadline_misses(svc) - m0 == misses


def test_svc_deadline_bounds_the_wait_behind_a_long_kernel(lib, svc):
    """The worker cannot start while another kernel holds every CU (tests/host/gpu_hog.hip: 160 KiB of
    LDS per CU for 600 ms).  A call then returns at its deadline (FECGPU_ERR_INVALID, counted as one
    withdrawal) instead of waiting for the long kernel, and the withdrawn request is never served: its
    repair rows are still untouched after the long kernel has ended and the queued worker has run."""
    import ctypes
    import os
    hog = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "host", "libgpuhog.so"))
    o = Oracle()
    k, r, L = 16, 4, 1200
    src = synth_bytes(k * L, 13).reshape(1, k, L)
    ts, _ = pinned(src)
    tr, hr = pinned(np.zeros((1, r, L), np.uint8))
    assert lib.fecgpu_block_svc_set_deadline(svc, 2000) == 0
    time.sleep(0.05)  # the worker has idled out: the next call must launch one
    m0 = lib.fecgpu_block_svc_deadline_misses(svc)
    assert hog.gpu_hog_launch(600) == 0
    time.sleep(0.02)  # the hog's workgroups are resident
    hr[:] = 0
    t0 = time.perf_counter()
    rc = lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr.data_ptr(), k, r, L, 21)
    dt = time.perf_counter() - t0
    assert rc == -1, "served while every CU was held: the test did not queue the worker"
    assert dt < 0.1, f"call waited {dt * 1e3:.1f} ms with a 2 ms deadline"
    assert lib.fecgpu_block_svc_deadline_misses(svc) - m0 == 1
    assert hog.gpu_hog_wait() == 0
    time.sleep(0.05)  # the queued worker ran, found nothing pending
    assert not hr.any(), "a withdrawn request was served"
    assert lib.fecgpu_block_svc_set_deadline(svc, 2000) == 0  # ends the back-off
    assert lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr.data_ptr(), k, r, L, 21) == 0
    assert np.array_equal(hr, o.rlc_encode_batch(src, r, 21))


def test_bulk_slices_yield_to_hooks_and_keep_the_bytes(lib, svc):
    """While the hooks are in use (a request within the last 100 ms), a zero-copy bulk call is cut into
    slices that start only when no hook request is pending (host_path.hip, Pacer); idle, it is one
    launch.  Either way the bytes are the device-resident engine's: encode with a block-number table,
    encode by row tables, and recover by row tables with per-repair seeds."""
    import ctypes as C
    from pquic_amd import Engine
    eng = Engine(0)
    k, r, L, nb = 16, 4, 1200, 1000  # 24 KB per block: 3 MiB slices of 131 blocks
    ctx = lib.fecgpu_host_ctx_create(0, 2, 64 << 20)
    assert ctx
    rng = np.random.default_rng(5)
    src = synth_bytes(nb * k * L, 77).reshape(nb, k, L)
    fbn = rng.integers(0, 1 << 24, nb).astype(np.uint32)
    ts, _ = pinned(src)
    tf, _ = pinned(fbn)
    want = torch.empty((nb, r, L), dtype=torch.uint8, device="cuda:0")
    eng.rlc_encode(ts.cuda(), want, k, r, L, fbn=tf.view(torch.int32).cuda())
    torch.cuda.synchronize()
    want = want.cpu().numpy()
    u64 = C.c_uint64
    lib.fecgpu_rlc_encode_rows_host.argtypes = [C.c_void_p] * 3 + [u64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]
    hook_src, _ = pinned(synth_bytes(k * L, 3).reshape(1, k, L))
    hook_rep, _ = pinned(np.zeros((1, r, L), np.uint8))

    def hooks_in_use():
        assert lib.fecgpu_block_svc_rlc_encode(svc, hook_src.data_ptr(), hook_rep.data_ptr(), k, r, L, 1) == 0

    st0 = eng.stats()
    for use_hooks in (False, True):
        time.sleep(0.15)  # no hook request in the last 100 ms
        if use_hooks:
            hooks_in_use()
        tr, hr = pinned(np.zeros((nb, r, L), np.uint8))
        assert lib.fecgpu_rlc_encode_host(ctx, ts.data_ptr(), tr.data_ptr(), nb, k, r, L, 0, tf.data_ptr()) == 0
        assert np.array_equal(hr, want), f"encode_host, hooks in use: {use_hooks}"
        # the same blocks by row tables (rows in the pinned buffers), repairs in reverse block order
        srows, _ = pinned((ts.data_ptr() + np.arange(nb * k, dtype=np.uint64) * L).astype(np.uint64))
        tr2, hr2 = pinned(np.zeros((nb, r, L), np.uint8))
        order = np.arange(nb)[::-1]
        rrows, _ = pinned((tr2.data_ptr() + ((order[:, None] * r + np.arange(r)[None, :]) * L).reshape(-1))
                          .astype(np.uint64))
        if use_hooks:
            hooks_in_use()
        assert lib.fecgpu_rlc_encode_rows_host(ctx, srows.data_ptr(), rrows.data_ptr(), nb, k, r, L,
                                               tf.data_ptr()) == 0
        assert np.array_equal(hr2[order], want), f"encode_rows_host, hooks in use: {use_hooks}"
        # recover by row tables: 4 erasures per block at rotating slots, seeds (fbn << 8) | i
        work = src.copy()
        sp = np.zeros((nb, 2), np.uint64)
        rp = np.zeros((nb, 2), np.uint64)
        for b in range(nb):
            miss = [(b + 3 * u) % k for u in range(4)]
            work[b, miss] = 0
            sp[b, 0] = ((1 << k) - 1) & ~sum(1 << m for m in set(miss))
            rp[b, 0] = (1 << r) - 1
        tw, hw = pinned(work)
        trep, _ = pinned(want)
        seeds = ((fbn.astype(np.uint64)[:, None] << 8) | np.arange(r, dtype=np.uint64)[None, :]).astype(np.uint32)
        tseed, _ = pinned(seeds)
        tsp, _ = pinned(sp.view(np.int64))
        trp, _ = pinned(rp.view(np.int64))
        tst, hst = pinned(np.full(nb, 0xEE, np.uint8))
        trec, hrec = pinned(np.zeros((nb, 2), np.int64))
        wrows, _ = pinned((tw.data_ptr() + np.arange(nb * k, dtype=np.uint64) * L).astype(np.uint64))
        prows, _ = pinned((trep.data_ptr() + np.arange(nb * r, dtype=np.uint64) * L).astype(np.uint64))
        if use_hooks:
            hooks_in_use()
        assert lib.fecgpu_rlc_decode_rows_host(ctx, wrows.data_ptr(), prows.data_ptr(), nb, k, r, L, tseed.data_ptr(),
                                               tsp.data_ptr(), trp.data_ptr(), tst.data_ptr(), trec.data_ptr()) == 0
        ok = hst == 0
        assert ok.sum() > nb * 0.9
        assert np.array_equal(hw[ok], src[ok]), f"decode_rows_host, hooks in use: {use_hooks}"
        st = eng.stats()
        if not use_hooks:
            assert st["yield_slices"] == st0["yield_slices"], "sliced while the hooks were idle"
    assert eng.stats()["yield_slices"] - st0["yield_slices"] >= 3 * 7, "no slicing while the hooks were in use"
    lib.fecgpu_host_ctx_destroy(ctx)
