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


# Deadline of the parity tests: generous, so that a request is never withdrawn because a fresh box was
# slow to start the worker.  The deadline tests set their own and restore this one.
SERVE_DEADLINE_US = 1_000_000


@pytest.fixture(scope="module")
def svc(lib):
    v = lib.fecgpu_block_svc_create(0)
    assert v
    assert lib.fecgpu_block_svc_set_deadline(v, SERVE_DEADLINE_US) == 0
    yield v
    lib.fecgpu_block_svc_destroy(v)


@pytest.fixture(scope="module")
def hog():
    import ctypes
    import os
    h = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "host", "libgpuhog.so"))
    yield h
    h.gpu_hog_release()


def hold_every_cu(hog):
    """Starts the hog and waits (a state, not a sleep) until all its workgroups are resident: then every
    CU's LDS is taken and no other kernel can start until the hog is released."""
    assert hog.gpu_hog_launch(5000) == 0
    t0 = time.perf_counter()
    while hog.gpu_hog_resident() < hog.gpu_hog_workgroups():
        assert hog.gpu_hog_running(), "the hog ended before all its workgroups were resident"
        assert time.perf_counter() - t0 < 4.0, "the hog's workgroups never all became resident"
        time.sleep(0.0005)


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


def _launches_after_idle(lib, svc):
    """Waits (for the state, bounded) until any worker of an earlier call has ended on its idle limit
    (20 ms without a request, worker clock) and returns the launch count."""
    t0 = time.perf_counter()
    while (st := lib.fecgpu_block_svc_worker_running(svc)) == 1:
        assert time.perf_counter() - t0 < 5.0, "the worker did not end on its idle limit"
        time.sleep(0.002)
    assert st == 0
    return lib.fecgpu_block_svc_launches(svc)


def test_svc_idle_exit_and_relaunch(lib, svc):
    """The worker ends after 20 ms without a request (and after 50 ms in all); the next call relaunches
    it and is served.  Back-to-back calls share one worker up to its lifetime: the count of launches is
    asserted only where the design fixes it, never against the box's speed."""
    o = Oracle()
    k, r, L = 16, 4, 1200
    src = synth_bytes(k * L, 7).reshape(1, k, L)
    ts, _ = pinned(src)
    tr, hr = pinned(np.zeros((1, r, L), np.uint8))
    want = o.rlc_encode_batch(src, r, 99)
    n0 = _launches_after_idle(lib, svc)
    t0 = time.perf_counter()
    assert lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr.data_ptr(), k, r, L, 99) == 0
    assert np.array_equal(hr, want)
    assert lib.fecgpu_block_svc_launches(svc) == n0 + 1  # no worker was running: this call launched one
    for _ in range(50):
        hr[:] = 0
        assert lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr.data_ptr(), k, r, L, 99) == 0
        assert np.array_equal(hr, want)
    n1 = lib.fecgpu_block_svc_launches(svc)
    if time.perf_counter() - t0 < 0.018:  # within one idle limit and the lifetime: the same worker served all
        assert n1 == n0 + 1
    n2 = _launches_after_idle(lib, svc)
    assert n2 == n1  # nothing ran while idle
    hr[:] = 0
    assert lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr.data_ptr(), k, r, L, 99) == 0
    assert np.array_equal(hr, want)
    assert lib.fecgpu_block_svc_launches(svc) == n2 + 1


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


def test_svc_deadline_withdraws_and_backs_off(lib, svc, hog):
    """A request no worker has claimed by the deadline is withdrawn.  Forced here, not raced: the hog
    holds every CU (all its workgroups resident, tests/host/gpu_hog.hip), so the worker cannot start.
    The call returns FECGPU_ERR_INVALID (the caller takes the launch path) at its deadline while the long
    kernel is still running, the withdrawal is counted once, the calls of the back-off return at once
    without posting, and no withdrawn request is ever served: its rows are still untouched after the hog
    is released and the worker has served a later request."""
    o = Oracle()
    k, r, L = 16, 4, 1200
    src = synth_bytes(k * L, 13).reshape(1, k, L)
    ts, _ = pinned(src)
    tr, hr = pinned(np.zeros((3, r, L), np.uint8))
    want = o.rlc_encode_batch(src, r, 21)
    m0 = lib.fecgpu_block_svc_deadline_misses(svc)
    assert lib.fecgpu_block_svc_set_deadline(svc, 2000) == 0
    try:
        hold_every_cu(hog)
        rc = lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr[0].data_ptr(), k, r, L, 21)
        assert rc == -1, "served while every CU was held"
        assert hog.gpu_hog_running(), "the call waited for the long kernel instead of its deadline"
        assert lib.fecgpu_block_svc_deadline_misses(svc) - m0 == 1
        # the back-off: the launch path at once (a call delayed past the back-off is withdrawn again)
        rc = lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr[1].data_ptr(), k, r, L, 21)
        assert rc == -1
        assert lib.fecgpu_block_svc_deadline_misses(svc) - m0 in (1, 2)
    finally:
        assert hog.gpu_hog_release() == 0
        assert lib.fecgpu_block_svc_set_deadline(svc, SERVE_DEADLINE_US) == 0  # also ends the back-off
    m1 = lib.fecgpu_block_svc_deadline_misses(svc)
    assert lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr[2].data_ptr(), k, r, L, 21) == 0
    assert np.array_equal(hr[2:3], want)
    assert not hr[:2].any(), "a withdrawn request was served"
    assert lib.fecgpu_block_svc_deadline_misses(svc) == m1


def test_svc_withdrawal_races_the_claim(lib, svc):
    """Deadline 0 against a running worker: the host's withdrawal (compare-and-swap on the request
    number, fine-grained mailbox) races the worker's claim on every call.  Whatever the interleaving,
    exactly one side wins: a call that returns OK has the oracle's bytes, a withdrawn one (-1, counted)
    left its rows untouched -- also after the worker has served later requests."""
    o = Oracle()
    k, r, L, n = 16, 4, 1200, 200
    src = synth_bytes(k * L, 17).reshape(1, k, L)
    ts, _ = pinned(src)
    tr, hr = pinned(np.zeros((n + 1, r, L), np.uint8))
    want = o.rlc_encode_batch(src, r, 33)
    assert lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr[n].data_ptr(), k, r, L, 33) == 0  # a worker runs
    m0 = lib.fecgpu_block_svc_deadline_misses(svc)
    rcs = []
    try:
        assert lib.fecgpu_block_svc_set_deadline(svc, 0) == 0
        for i in range(n):
            rc = lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr[i].data_ptr(), k, r, L, 33)
            assert rc in (0, -1)
            rcs.append(rc)
            if rc == -1:
                assert lib.fecgpu_block_svc_set_deadline(svc, 0) == 0  # ends the back-off: race again
    finally:
        assert lib.fecgpu_block_svc_set_deadline(svc, SERVE_DEADLINE_US) == 0
    withdrawn = [i for i in range(n) if rcs[i] == -1]
    assert lib.fecgpu_block_svc_deadline_misses(svc) - m0 == len(withdrawn)
    hr[n] = 0
    assert lib.fecgpu_block_svc_rlc_encode(svc, ts.data_ptr(), tr[n].data_ptr(), k, r, L, 33) == 0
    assert np.array_equal(hr[n:], want)
    for i in range(n):
        if rcs[i] == 0:
            assert np.array_equal(hr[i:i + 1], want), f"call {i}: served with the wrong bytes"
        else:
            assert not hr[i].any(), f"call {i}: withdrawn and served"


def test_bulk_slices_yield_to_hooks_and_keep_the_bytes(lib, svc):
    """While the hooks are in use (a request within the last yield_window_ms), a zero-copy bulk call is
    cut into slices (host_path.hip, Pacer); idle, it is one launch.  Either way the bytes are the
    device-resident engine's: encode with a block-number table, by consecutive numbers from fbn_base
    (each slice starts at its own block number), by row tables with and without fbn[], and recover by
    row tables with per-repair seeds.  The test never races the window: the idle leg starts well after
    the last request, and the hooked leg stretches the window to minutes (knob yield_window_ms)."""
    import ctypes as C
    from pquic_amd import Engine
    eng = Engine(0)
    k, r, L, nb = 16, 4, 1200, 1000  # 24 KB per block: 2.25 MiB slices of 98 blocks
    FB0 = (1 << 24) - 300  # block numbers wrap inside the batch
    ctx = lib.fecgpu_host_ctx_create(0, 2, 64 << 20)
    assert ctx
    rng = np.random.default_rng(5)
    src = synth_bytes(nb * k * L, 77).reshape(nb, k, L)
    fbn = rng.integers(0, 1 << 24, nb).astype(np.uint32)
    ts, _ = pinned(src)
    tf, _ = pinned(fbn)
    dsrc = ts.cuda()

    def device_encode(fbn_base=0, table=None):
        out = torch.empty((nb, r, L), dtype=torch.uint8, device="cuda:0")
        eng.rlc_encode(dsrc, out, k, r, L, fbn_base=fbn_base, fbn=table)
        torch.cuda.synchronize()
        return out.cpu().numpy()
    want = device_encode(table=tf.view(torch.int32).cuda())
    want_seq = device_encode(fbn_base=FB0)
    want_zero = device_encode()
    # the device path itself against the oracle on a sample of blocks (both numberings)
    o = Oracle()
    for b in (0, 299, 300, nb - 1):
        assert np.array_equal(want[b:b + 1], o.rlc_encode_batch(src[b:b + 1], r, int(fbn[b])))
        assert np.array_equal(want_seq[b:b + 1], o.rlc_encode_batch(src[b:b + 1], r, (FB0 + b) & 0xffffff))
        assert np.array_equal(want_zero[b:b + 1], o.rlc_encode_batch(src[b:b + 1], r, b))
    u64 = C.c_uint64
    lib.fecgpu_rlc_encode_rows_host.argtypes = [C.c_void_p] * 3 + [u64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]
    hook_src, _ = pinned(synth_bytes(k * L, 3).reshape(1, k, L))
    hook_rep, _ = pinned(np.zeros((1, r, L), np.uint8))
    srows, _ = pinned((ts.data_ptr() + np.arange(nb * k, dtype=np.uint64) * L).astype(np.uint64))
    order = np.arange(nb)[::-1]  # repairs by row table in reverse block order

    def hooks_in_use():
        assert lib.fecgpu_block_svc_rlc_encode(svc, hook_src.data_ptr(), hook_rep.data_ptr(), k, r, L, 1) == 0

    st0 = eng.stats()
    window0 = eng.get_knob("yield_window_ms")
    try:
        for use_hooks in (False, True):
            if use_hooks:
                eng.set_knob("yield_window_ms", 600000)
                hooks_in_use()
            else:
                time.sleep(2 * window0 / 1000)  # no hook request within the window
            tag = f"hooks in use: {use_hooks}"
            tr, hr = pinned(np.zeros((nb, r, L), np.uint8))
            assert lib.fecgpu_rlc_encode_host(ctx, ts.data_ptr(), tr.data_ptr(), nb, k, r, L, 0, tf.data_ptr()) == 0
            assert np.array_equal(hr, want), f"encode_host with fbn[], {tag}"
            hr[:] = 0
            assert lib.fecgpu_rlc_encode_host(ctx, ts.data_ptr(), tr.data_ptr(), nb, k, r, L, FB0, None) == 0
            assert np.array_equal(hr, want_seq), f"encode_host from fbn_base, {tag}"
            for table, expect in ((tf.data_ptr(), want), (None, want_zero)):
                tr2, hr2 = pinned(np.zeros((nb, r, L), np.uint8))
                rrows, _ = pinned((tr2.data_ptr() + ((order[:, None] * r + np.arange(r)[None, :]) * L).reshape(-1))
                                  .astype(np.uint64))
                assert lib.fecgpu_rlc_encode_rows_host(ctx, srows.data_ptr(), rrows.data_ptr(), nb, k, r, L,
                                                       table) == 0
                assert np.array_equal(hr2[order], expect), f"encode_rows_host, fbn[]: {table is not None}, {tag}"
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
            assert lib.fecgpu_rlc_decode_rows_host(ctx, wrows.data_ptr(), prows.data_ptr(), nb, k, r, L,
                                                   tseed.data_ptr(), tsp.data_ptr(), trp.data_ptr(), tst.data_ptr(),
                                                   trec.data_ptr()) == 0
            ok = hst == 0
            assert ok.sum() > nb * 0.9
            assert np.array_equal(hw[ok], src[ok]), f"decode_rows_host, {tag}"
            st = eng.stats()
            if not use_hooks:
                assert st["yield_slices"] == st0["yield_slices"], "sliced while the hooks were idle"
        # 11 slices per call (98 blocks each): five calls
        assert eng.stats()["yield_slices"] - st0["yield_slices"] >= 5 * 10, "no slicing while the hooks were in use"
    finally:
        eng.set_knob("yield_window_ms", window0)
    lib.fecgpu_host_ctx_destroy(ctx)
