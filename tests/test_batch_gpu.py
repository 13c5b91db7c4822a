"""Batching adapter (include/pquic_fec_batch.h): blocks from many "connections" queued into
GPU batches, completed through callbacks.  A batched block must end in exactly the state the
synchronous protocol operation leaves it in, so every case is checked against the fixtures the
reference pluglets produced (the same ones tests/test_protoops_gpu.py uses), with batches that
mix symbol lengths, block numbers and flush causes (full, deadline, drain)."""
import ctypes as C
import os
import time

import numpy as np
import pytest

from golden_io import decode_sources, encode_inputs, load, load_npz, sha, window_inputs
from oracle_py import Oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
# PQUIC_TEST_MINIHOST: a sanitizer build over the CPU engine stand-in (tests/sanitize, test_sanitize.py)
MINIHOST = os.environ.get("PQUIC_TEST_MINIHOST") or os.path.join(ROOT, "tests", "host", "libminihost.so")


def _p(a, t=C.c_uint8):
    return a.ctypes.data_as(C.POINTER(t))


class Batch:
    def __init__(self, batch_blocks, max_delay_us=1000, max_symbol=9000, nstreams=2, arena=False, poll_blocks=0,
                 arena_bytes=256 << 20, connections=0, conn_bytes=1 << 20):
        L = C.CDLL(MINIHOST)
        L.mh_arena_enable.argtypes = [C.c_size_t]
        for f in ("mh_batch_generate", "mh_batch_recover", "mh_batch_status", "mh_live_allocations"):
            getattr(L, f).restype = C.c_long
        L.mh_batch_generate.argtypes = [C.c_int, C.c_uint32, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                                        C.c_uint64]
        L.mh_batch_recover.argtypes = [C.c_int, C.c_uint32, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_uint64]
        L.mh_batch_status.argtypes = [C.c_long, C.POINTER(C.c_int)]
        L.mh_batch_repairs.argtypes = [C.c_long, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.mh_batch_recovered.argtypes = [C.c_long, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_int),
                                         C.c_void_p]
        L.mh_batch_poll.argtypes = [C.c_uint64]
        L.mh_stream_open.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_uint32]
        L.mh_batch_generate_window.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64]
        L.mh_batch_generate_window.restype = C.c_long
        L.mh_batch_connections.argtypes = [C.c_int, C.c_size_t]
        L.mh_batch_order.argtypes = [C.c_long]
        L.mh_batch_order.restype = C.c_long
        L.mh_arena_live.argtypes = [C.c_int]
        L.mh_arena_live.restype = C.c_long
        self.L = L
        self.stream_stride = {}
        assert L.mh_bind(0) == 0
        self.base = L.mh_live_allocations()
        if arena:  # symbols in a plugin-style arena the batcher gathers rows from (registered heap)
            assert L.mh_arena_enable(arena_bytes) == 0
        assert L.mh_batch_open(0, batch_blocks, max_delay_us, max_symbol, nstreams, poll_blocks) == 0
        if arena:
            assert L.mh_batch_register_arena() == 0
        if connections:  # connections with arenas of their own, each registered (one per plugin instance)
            assert L.mh_batch_connections(connections, conn_bytes) == 0
        self.meta = {}

    def use(self, conn):
        """Build and submit the next blocks on connection `conn` (-1: the default one)."""
        assert self.L.mh_batch_use_connection(conn) == 0

    def generate(self, xor, fbn, srcs, r, now=0):
        k = len(srcs)
        stride = max([len(s) for s in srcs] + [1])
        buf = np.zeros((k, stride), np.uint8)
        lens = np.zeros(k, np.uint16)
        for j, s in enumerate(srcs):
            buf[j, : len(s)] = s
            lens[j] = len(s)
        t = self.L.mh_batch_generate(int(xor), fbn, k, r, buf.ctypes.data, lens.ctypes.data, stride, now)
        assert t >= 0
        self.meta[t] = (k, r, stride)
        return t

    def open_stream(self, syms, first_fpid=0):
        """A window sender's symbols (one connection); window blocks point into it."""
        stride = max(len(x) for x in syms)
        buf = np.zeros((len(syms), stride), np.uint8)
        lens = np.array([len(x) for x in syms], np.uint16)
        for j, x in enumerate(syms):
            buf[j, : len(x)] = x
        sid = self.L.mh_stream_open(len(syms), buf.ctypes.data, lens.ctypes.data, stride, first_fpid)
        assert sid >= 0
        self.stream_stride[sid] = stride
        return sid

    def generate_window(self, sid, start, k, r, now=0):
        t = self.L.mh_batch_generate_window(sid, start, k, r, now)
        assert t >= 0
        self.meta[t] = (k, r, self.stream_stride[sid])
        return t

    def recover(self, xor, fbn, srcs, reps, fpids, now=0):
        k, r = len(srcs), len(reps)
        stride = max([len(s) for s in srcs + reps if s is not None] + [1])
        sb = np.zeros((k, stride), np.uint8)
        sl = np.zeros(k, np.uint16)
        spres = np.zeros(k, np.uint8)
        for j, s in enumerate(srcs):
            if s is not None:
                sb[j, : len(s)] = s
                sl[j] = len(s)
                spres[j] = 1
        rb = np.zeros((max(r, 1), stride), np.uint8)
        rl = np.zeros(max(r, 1), np.uint16)
        rpres = np.zeros(max(r, 1), np.uint8)
        for i, s in enumerate(reps):
            if s is not None:
                rb[i, : len(s)] = s
                rl[i] = len(s)
                rpres[i] = 1
        fp = np.zeros(max(r, 1), np.uint64)
        fp[:r] = fpids
        t = self.L.mh_batch_recover(int(xor), fbn, k, r, sb.ctypes.data, sl.ctypes.data, spres.ctypes.data, stride,
                                    rb.ctypes.data, rl.ctypes.data, rpres.ctypes.data, fp.ctypes.data, stride, now)
        assert t >= 0
        self.meta[t] = (k, r, stride)
        return t

    def status(self, t):
        calls = C.c_int(0)
        ret = self.L.mh_batch_status(t, C.byref(calls))
        return ret, calls.value

    def repairs(self, t):
        k, r, stride = self.meta[t]
        rep = np.zeros((max(r, 1), stride), np.uint8)
        rl = np.zeros(max(r, 1), np.uint16)
        fp = np.zeros(max(r, 1), np.uint64)
        self.L.mh_batch_repairs(t, rep.ctypes.data, rl.ctypes.data, fp.ctypes.data, stride)
        return [rep[i, : rl[i]].copy() for i in range(r)], [int(x) for x in fp[:r]]

    def recovered(self, t):
        k, r, stride = self.meta[t]
        out = np.zeros((k, stride), np.uint8)
        ol = np.zeros(k, np.uint16)
        rec = np.zeros(k, np.uint8)
        cur = C.c_int(0)
        ofp = np.zeros(k, np.uint32)
        self.L.mh_batch_recovered(t, out.ctypes.data, ol.ctypes.data, rec.ctypes.data, stride, C.byref(cur),
                                  ofp.ctypes.data)
        self.last_fpids = {j: int(ofp[j]) for j in range(k) if rec[j]}
        return {j: out[j, : ol[j]].copy() for j in range(k) if rec[j]}, cur.value

    def stats(self):
        s = (C.c_uint64 * 15)()
        self.L.mh_batch_get_stats(s)
        keys = ["submitted", "completed", "batches", "flushed_full", "flushed_deadline", "flushed_drain",
                "immediate", "engine_errors", "windows", "window_rows", "rows_in_place", "rows_staged",
                "jobs_allocated", "job_alloc_us", "deadline_holds"]
        return dict(zip(keys, list(s)))

    def close(self):
        self.L.mh_batch_close()
        assert self.L.mh_live_allocations() == self.base, "blocks or symbols leaked"


def _encode_jobs():
    """(xor, fbn, sources, r, expected repair hex or sha, fpids, ret) for every fixture case."""
    e = load("encode_cases.json")
    full = load_npz("encode_full.npz")  # noqa: F841  (encode_inputs reads it)
    jobs = []
    for case in e["varlen"]:
        srcs = [np.frombuffer(bytes.fromhex(h), np.uint8) for h in case["src_hex"]]
        jobs.append((case["scheme"] == "xor", case["fbn"], srcs, case["r"], ("hex", case["rep_hex"]),
                     case["repair_fpid_raw"], case["ret"]))
    for case in e["cases"]:
        if case["k"] > 100 or case["r"] > 100:
            continue
        src = encode_inputs(case)
        for b in range(case["nblocks"]):
            fbn = (case["fbn_base"] + b) & 0xFFFFFF
            jobs.append((case["scheme"] == "xor", fbn, list(src[b]), case["r"], ("sha", case["block_sha256"][b]),
                         case["repair_fpid_raw"][b], 0))
    for p in e["preconditions"]:
        srcs = [np.arange(10, dtype=np.uint8) + j for j in range(p["k"])]
        jobs.append((p["scheme"] == "xor", 3, srcs, p["r"], None, None, p["ret"]))
    return jobs


def _check_generate(bt, t, job):
    xor, fbn, srcs, r, want, fpids, ret = job
    got_ret, calls = bt.status(t)
    assert calls == 1 and got_ret == ret
    if want is None:
        return
    reps, fps = bt.repairs(t)
    if want[0] == "hex":
        assert [x.tobytes().hex() for x in reps] == want[1]
    else:
        assert sha(np.stack(reps).tobytes()) == want[1]
    assert fps == fpids


@pytest.mark.parametrize("poll_blocks", [1, 3, 7])
def test_batch_bounded_poll(poll_blocks):
    """cfg.poll_blocks: each poll completes at most that many blocks, a batch's completions spread over
    several polls; every block completes once, with the reference's results."""
    import time
    bt = Batch(4, poll_blocks=poll_blocks)
    jobs = [j for j in _encode_jobs() if j[4] is not None][:23]
    tickets = [bt.generate(*j[:4], now=i) for i, j in enumerate(jobs)]
    bt.L.mh_batch_poll(10 ** 9)  # flushes the part-filled queue (past its deadline)
    order, t0 = [], time.time()
    while len(order) < len(tickets) and time.time() - t0 < 30:
        n = bt.L.mh_batch_poll(10 ** 9)
        assert 0 <= n <= poll_blocks
        order += [t for t in tickets if t not in order and bt.status(t)[1] == 1]
        if not n:
            time.sleep(0.001)
    assert sorted(order) == sorted(tickets), "every block completes"
    for t, j in zip(tickets, jobs):
        _check_generate(bt, t, j)
    assert bt.L.mh_batch_drain() == 0
    bt.close()


@pytest.mark.parametrize("batch_blocks", [1, 5, 64])
def test_batch_generate_matches_reference(batch_blocks):
    bt = Batch(batch_blocks)
    jobs = _encode_jobs()
    tickets = [bt.generate(*j[:4], now=i) for i, j in enumerate(jobs)]
    bt.L.mh_batch_drain()
    for t, j in zip(tickets, jobs):
        _check_generate(bt, t, j)
    st = bt.stats()
    assert st["completed"] + st["immediate"] == len(jobs) == st["submitted"] + st["immediate"]
    assert st["engine_errors"] == 0
    bt.close()


@pytest.mark.parametrize("batch_blocks,max_symbol", [(5, 9000), (64, 1200), (64, 9000)])
def test_batch_generate_gathers_from_registered_arena(batch_blocks, max_symbol):
    """With the symbols' arena registered (pquic_fec_batch_register_heap), RLC generate batches read
    the sources and write the repairs in place (fecgpu_rlc_encode_rows); rows outside the arena
    (symbols > 2092 B), shorter than the block (zero-padded) or repairs shorter than the stride are
    staged.  Same repairs, FPIDs and return values as the reference fixtures; no leaks."""
    bt = Batch(batch_blocks, max_symbol=max_symbol, arena=True)
    jobs = [j for j in _encode_jobs() if max(len(s) for s in j[2]) <= max_symbol]
    # blocks whose rows are all exactly max_symbol long: sources and repairs both in place
    rng = np.random.default_rng(max_symbol + batch_blocks)
    o = Oracle()
    for b in range(40):
        k, r = int(rng.integers(1, 33)), int(rng.integers(1, 9))
        srcs = [rng.integers(0, 256, max_symbol, dtype=np.uint8) for _ in range(k)]
        fbn = int(rng.integers(0, 1 << 24))
        rep = o.rlc_encode_batch(np.stack(srcs)[None], r, fbn)[0]
        jobs.append((False, fbn, srcs, r, ("hex", [x.tobytes().hex() for x in rep]),
                     [(fbn << 8) | i for i in range(r)], 0))
    tickets = [bt.generate(*j[:4], now=i) for i, j in enumerate(jobs)]
    bt.L.mh_batch_drain()
    for t, j in zip(tickets, jobs):
        _check_generate(bt, t, j)
    st = bt.stats()
    assert st["engine_errors"] == 0
    bt.close()


@pytest.mark.parametrize("conns", [0, 2])
def test_batch_small_jobs_keep_the_bytes(conns):
    """batch_blocks >= 1024: a job the caller has to allocate itself (no idle one, no spare from the
    provisioner) is a small one, batch_blocks / 16 blocks (batch.c job_get), flushed at its own capacity.
    A fresh batcher's first job is always one.  600 k16 r4 blocks generated back to back (fewer than
    batch_blocks, so any full flush is a small job's), then recovered with 4 erasures each: repairs and
    recovered rows equal the oracle's, staged (conns 0) and in place (conns 2)."""
    o = Oracle()
    k, r, L, n = 16, 4, 1200, 600
    rng = np.random.default_rng(77 + conns)
    src = rng.integers(0, 256, (n, k, L), dtype=np.uint8)
    fbn0 = int(rng.integers(0, 1 << 24))
    want = o.rlc_encode_batch(src, r, fbn0)
    bt = Batch(1024, max_symbol=L, connections=conns, conn_bytes=16 << 20)
    tickets = []
    for b in range(n):
        if conns:
            bt.use(b % conns)
        tickets.append(bt.generate(False, (fbn0 + b) & 0xFFFFFF, list(src[b]), r, now=b))
    bt.L.mh_batch_drain()
    st = bt.stats()
    assert st["engine_errors"] == 0 and st["completed"] == n
    assert st["flushed_full"] >= 1, "no job was flushed below batch_blocks: no small job ran"
    for b, t in enumerate(tickets):
        assert bt.status(t) == (0, 1)
        reps, fps = bt.repairs(t)
        assert np.array_equal(np.stack(reps), want[b]), b
        assert fps == [(((fbn0 + b) & 0xFFFFFF) << 8) | i for i in range(r)]
    miss = [rng.choice(k, 4, replace=False) for _ in range(n)]
    tickets = []
    for b in range(n):
        fbn = (fbn0 + b) & 0xFFFFFF
        srcs = [None if j in miss[b] else src[b, j] for j in range(k)]
        tickets.append(_recover_on(bt, conns, b, False, fbn, srcs, list(want[b]),
                                   [(fbn << 8) | i for i in range(r)], now=n + b))
    bt.L.mh_batch_drain()
    assert bt.stats()["engine_errors"] == 0
    nrec = 0
    for b, t in enumerate(tickets):
        ret, calls = bt.status(t)
        assert calls == 1 and ret == 0
        rec, _ = bt.recovered(t)
        fbn = (fbn0 + b) & 0xFFFFFF
        _, out = o.rlc_decode_block(fbn, [None if j in miss[b] else src[b, j] for j in range(k)], list(want[b]))
        assert sorted(rec) == sorted(out), b  # none where the reference would crash (about 1 %)
        for j, row in rec.items():
            assert np.array_equal(row, src[b, j]) and np.array_equal(row, out[j]), (b, j)
        nrec += len(rec)
    assert nrec >= 0.95 * 4 * n
    bt.close()


def test_batch_small_jobs_across_shapes():
    """Jobs reused across block shapes (batch_blocks >= 1024, where job_get also takes a job that only holds
    a small one's worth of a shape): a job's capacity for a shape is what its row buffers hold (batch.c
    job_prepare).  First 2100 k4 r1 blocks (full-size k4 jobs, idle after the drain), then 600 k32 r8 blocks
    (a full k4 job holds 128 of them, not 1024), then the shapes interleaved block by block; repairs equal
    the oracle's (and under ASan, test_sanitize.py, no row lands past a buffer)."""
    o = Oracle()
    L = 1200
    rng = np.random.default_rng(11)
    shapes = [(4, 1), (32, 8), (16, 4), (8, 2)]
    bt = Batch(1024, max_symbol=L)
    tickets = []
    order = [(4, 1)] * 2100 + [None] + [(32, 8)] * 600 + [None] + \
        [shapes[(b * 7 + b // 5) % len(shapes)] for b in range(480)]
    for b, shape in enumerate(order):
        if shape is None:
            bt.L.mh_batch_drain()
            continue
        k, r = shape
        src = rng.integers(0, 256, (1, k, L), dtype=np.uint8)
        fbn = int(rng.integers(0, 1 << 24))
        tickets.append((bt.generate(False, fbn, list(src[0]), r, now=b), o.rlc_encode_batch(src, r, fbn)[0]))
        if b > 2702 and b % 40 == 39:  # deadline flushes in the interleaved part only
            bt.L.mh_batch_poll(10 ** 9)
    bt.L.mh_batch_drain()
    st = bt.stats()
    assert st["engine_errors"] == 0 and st["completed"] == len(tickets)
    for t, want in tickets:
        assert bt.status(t) == (0, 1)
        reps, _ = bt.repairs(t)
        assert np.array_equal(np.stack(reps), want)
    bt.close()


@pytest.mark.skipif(bool(os.environ.get("PQUIC_TEST_MINIHOST")), reason="stalls the GPU (no GPU under the CPU stand-in)")
def test_batch_deadline_holds_behind_a_stalled_gpu():
    """While the GPU is stalled (a kernel holds every CU, tests/host/libgpuhog.so), blocks keep arriving
    and every poll finds their queue overdue.  With two jobs in flight and none idle, the overdue queue
    stays open and keeps filling (pquic_fec_batch_stats_t deadline_holds) instead of being flushed into a
    batch whose successor the caller would have to page-lock on its own thread, which waits out the stall.
    Asserted: at most one job allocated by the caller during the stall; some polls held the queue (and
    fewer batches than blocks were flushed), unless the provisioner had a job ready for every flush; every
    block's repairs equal the oracle's once the GPU is released."""
    hog = C.CDLL(os.path.join(ROOT, "tests", "host", "libgpuhog.so"))
    o = Oracle()
    k, r, L, n = 16, 4, 1200, 40
    rng = np.random.default_rng(5)
    src = rng.integers(0, 256, (n + 1, k, L), dtype=np.uint8)
    want = o.rlc_encode_batch(src, r, 1000)
    bt = Batch(64, max_delay_us=100, max_symbol=L)
    tickets = [bt.generate(False, 1000, list(src[0]), r, now=0)]  # warm-up: one job, completed
    bt.L.mh_batch_drain()
    s0 = bt.stats()
    try:
        assert hog.gpu_hog_launch(5000) == 0
        t0 = time.perf_counter()
        while hog.gpu_hog_resident() < hog.gpu_hog_workgroups():
            assert hog.gpu_hog_running() and time.perf_counter() - t0 < 4.0
            time.sleep(0.0005)
        now = 10_000
        for b in range(1, n + 1):
            tickets.append(bt.generate(False, 1000 + b, list(src[b]), r, now=now))
            now += 1000  # every poll finds the queue overdue
            bt.L.mh_batch_poll(now)
        s1 = bt.stats()
    finally:
        assert hog.gpu_hog_release() == 0
    bt.L.mh_batch_drain()
    st = bt.stats()
    assert st["completed"] == n + 1 and st["engine_errors"] == 0
    assert s1["jobs_allocated"] - s0["jobs_allocated"] <= 1, (s0, s1)
    held = s1["deadline_holds"] - s0["deadline_holds"]
    flushed = s1["flushed_deadline"] - s0["flushed_deadline"]
    assert held > 0 or flushed == n, (s0, s1)  # held, or the provisioner kept a job ready for every flush
    if held:
        assert flushed < n
    for b, t in enumerate(tickets):
        assert bt.status(t) == (0, 1)
        reps, _ = bt.repairs(t)
        assert np.array_equal(np.stack(reps), want[b]), b
    bt.close()


def _decode_jobs():
    d = load("decode_cases.json")
    o = Oracle()
    jobs = []
    for case in d["cases"] + d["zero_cases"] + d["varlen_cases"]:
        if case["k"] > 100:
            continue
        srcs_full = decode_sources(case)
        k, r, fbn = case["k"], case["r"], case["fbn"]
        if case["scheme"] == "xor":
            reps_full = [o.xor_encode_block(srcs_full)[1]]
            fpids = [fbn << 8]
        else:
            reps_full = o.rlc_encode_block(fbn, srcs_full, r)[1]
            fpids = [(fbn << 8) | i for i in range(r)]
        srcs = [None if j in case["src_missing"] else srcs_full[j] for j in range(k)]
        reps = [reps_full[i] if i in case["rep_present"] else None for i in range(r)]
        jobs.append((case, srcs, reps, fpids))
    return jobs


def _recover_on(bt, conns, i, *args, now=0):
    """bt.recover on connection i % conns (its own registered arena: the gather path), or on the
    default connection (no arena registered: rows staged) when conns is 0."""
    if conns:
        bt.use(i % conns)
    return bt.recover(*args, now=now)


@pytest.mark.parametrize("conns", [0, 3])
@pytest.mark.parametrize("batch_blocks", [3, 128])
def test_batch_recover_matches_reference(batch_blocks, conns):
    """Every reference decode fixture (crash patterns included) through the batcher, rows staged
    (conns 0) or read and written in place in per-connection arenas (conns 3)."""
    # the gather path reads rows in place only at the batch stride: 1200-B cases (the others stay
    # covered staged, conns 0)
    bt = Batch(batch_blocks, max_symbol=1200 if conns else 9000, connections=conns, conn_bytes=16 << 20)
    jobs = [j for j in _decode_jobs() if not conns or max([len(x) for x in j[1] + j[2] if x is not None] + [1]) <= 1200]
    tickets = [_recover_on(bt, conns, i, c["scheme"] == "xor", c["fbn"], s, r, f, now=i)
               for i, (c, s, r, f) in enumerate(jobs)]
    bt.L.mh_batch_drain()
    n = 0
    for t, (case, srcs, _, _) in zip(tickets, jobs):
        ret, calls = bt.status(t)
        assert calls == 1, case["tag"]
        rec, cur = bt.recovered(t)
        if case["crashed"]:  # the reference segfaults here; the adapter recovers nothing
            assert ret == 0 and rec == {}
            continue
        assert ret == case["ret"], case["tag"]
        assert {str(j): sha(v.tobytes()) for j, v in sorted(rec.items())} == case["recovered"], case["tag"]
        assert {str(j): len(v) for j, v in rec.items()} == case["recovered_len"]
        present = sum(s is not None for s in srcs)
        assert cur == (present + len(rec) if case["scheme"] == "rlc" else present)
        n += 1
    assert n > (200 if conns else 350)
    if conns:
        assert bt.stats()["rows_in_place"] > 1000
    bt.close()


def test_batch_deadline_flush():
    """A queue below batch_blocks is flushed by poll once its oldest block is max_delay_us old."""
    bt = Batch(1000, max_delay_us=100)
    srcs = [np.full(1200, j, np.uint8) for j in range(16)]
    tickets = [bt.generate(False, 7 + i, srcs, 4, now=10) for i in range(3)]
    assert bt.L.mh_batch_poll(50) == 0  # 40 us old: not due
    assert all(bt.status(t)[0] == -1 for t in tickets)
    done = bt.L.mh_batch_poll(110)  # due: flushed to the worker
    deadline = time.time() + 30
    while done < 3 and time.time() < deadline:
        time.sleep(0.001)
        done += bt.L.mh_batch_poll(110)
    assert done == 3
    st = bt.stats()
    assert st["flushed_deadline"] == 1 and st["batches"] == 1
    o = Oracle()
    for i, t in enumerate(tickets):
        assert bt.status(t) == (0, 1)
        reps, fps = bt.repairs(t)
        want = o.rlc_encode_block(7 + i, srcs, 4)[1]
        assert all((a == b).all() for a, b in zip(reps, want))
        assert fps == [((7 + i) << 8) | j for j in range(4)]
    bt.close()


def test_batch_mixed_keys_and_symbol_cap():
    """Blocks of different (scheme, k, r) go to separate queues; a symbol above max_symbol is
    refused without a callback."""
    bt = Batch(4, max_symbol=1500)
    o = Oracle()
    jobs = []
    rng = np.random.default_rng(5)
    for i in range(40):
        k, r = [(4, 1), (16, 4), (8, 2), (32, 8)][i % 4]
        xor = (k, r) == (4, 1) and i % 8 == 0
        srcs = [rng.integers(0, 256, int(rng.integers(1, 1500)), dtype=np.uint8) for _ in range(k)]
        jobs.append((xor, 100 + i, srcs, r, bt.generate(xor, 100 + i, srcs, r, now=i)))
    big = [np.zeros(1600, np.uint8)] * 4
    k = len(big)
    buf = np.zeros((k, 1600), np.uint8)
    lens = np.full(k, 1600, np.uint16)
    assert bt.L.mh_batch_generate(0, 1, k, 2, buf.ctypes.data, lens.ctypes.data, 1600, 0) == -1
    bt.L.mh_batch_drain()
    for xor, fbn, srcs, r, t in jobs:
        assert bt.status(t) == (0, 1)
        reps, _ = bt.repairs(t)
        L = max(len(s) for s in srcs)
        pad = [np.pad(s, (0, L - len(s))) for s in srcs]
        want = [o.xor_encode_block(pad)[1]] if xor else o.rlc_encode_block(fbn, pad, r)[1]
        assert all(a.tobytes() == b.tobytes() for a, b in zip(reps, want))
    bt.close()


@pytest.mark.parametrize("conns", [0, 3])
@pytest.mark.parametrize("batch_blocks", [4, 64])
def test_batch_recover_window_framework_blocks(batch_blocks, conns):
    """The batcher on window-framework-shaped blocks (window_cases.json): block numbered by its
    window start, repairs seeded by their own FPIDs (block number 0, or mixed), mixed in one
    queue with block-framework blocks of the same (k, r); rows staged (conns 0) or on the gather
    path in per-connection arenas (conns 3)."""
    bt = Batch(batch_blocks, max_symbol=1200 if conns else 9000, connections=conns, conn_bytes=16 << 20)
    o = Oracle()
    d = load("window_cases.json")
    jobs = []
    for i, case in enumerate(d["cases"]):
        srcs_full, reps_full, fpids = window_inputs(case, o)
        if conns and max(len(x) for x in srcs_full + reps_full) > 1200:
            continue
        k, r = case["k"], case["r"]
        srcs = [None if j in case["src_missing"] else srcs_full[j] for j in range(k)]
        reps = [reps_full[i2] if i2 in case["rep_present"] else None for i2 in range(r)]
        jobs.append((case, srcs, _recover_on(bt, conns, i, case["scheme"] == "xor", case["fbn"], srcs, reps, fpids,
                                             now=i)))
    bt.L.mh_batch_drain()
    n = 0
    for case, srcs, t in jobs:
        ret, calls = bt.status(t)
        assert calls == 1, case["tag"]
        rec, cur = bt.recovered(t)
        if case["crashed"]:
            assert ret == 0 and rec == {}
            continue
        assert ret == case["ret"], case["tag"]
        assert {str(j): sha(v.tobytes()) for j, v in sorted(rec.items())} == case["recovered"], case["tag"]
        assert {str(j): f for j, f in bt.last_fpids.items()} == case["recovered_fpid"], case["tag"]
        present = sum(s is not None for s in srcs)
        assert cur == (present + len(rec) if case["scheme"] == "rlc" else present)
        n += 1
    assert n > (60 if conns else 150)
    if conns:
        assert bt.stats()["rows_in_place"] > 200
    bt.close()


@pytest.mark.parametrize("fail_at", [0, 1, 2, 5, 7])
def test_batch_generate_allocation_failure_matches_sync(fail_at):
    """An allocator failure during generate (the fail_at-th allocation of the operation; a repair
    takes two, struct then data) ends a batched block exactly as the synchronous operation ends
    it: same return value (PICOQUIC_ERROR_MEMORY), the same repairs attached with the same bytes
    and FPIDs, and nothing leaked (rlc_fec_scheme_generate_gf256.c:50-70 allocates per repair)."""
    rng = np.random.default_rng(11 + fail_at)
    k, r, fbn = 16, 4, 321
    srcs = [rng.integers(0, 256, 1200, dtype=np.uint8) for _ in range(k)]
    buf = np.stack(srcs)
    lens = np.full(k, 1200, np.uint16)
    bt = Batch(1)
    bt.L.mh_fail_next_generate.argtypes = [C.c_long]
    bt.L.mh_fail_alloc_after.argtypes = [C.c_long]
    # synchronous protocol operation with the failure injected
    rep = np.zeros((r, 1200), np.uint8)
    rl = np.zeros(r, np.uint16)
    fp = np.zeros(r, np.uint64)
    sch = np.zeros(2, np.uint64)
    bt.L.mh_generate.restype = C.c_long
    bt.L.mh_fail_next_generate(fail_at)
    ret_sync = bt.L.mh_generate(0, fbn, k, r, _p(buf), _p(lens, C.c_uint16), 1200, _p(rep), _p(rl, C.c_uint16),
                                _p(fp, C.c_uint64), 1200, _p(sch, C.c_uint64))
    # the batched block with the same failure
    bt.L.mh_fail_next_generate(fail_at)
    t = bt.generate(False, fbn, srcs, r)
    bt.L.mh_batch_drain()
    bt.L.mh_fail_alloc_after(-1)
    ret_b, calls = bt.status(t)
    assert ret_sync == 0x405 and (ret_b, calls) == (ret_sync, 1)
    reps_b, fps_b = bt.repairs(t)
    n = fail_at // 2  # repairs fully allocated before the failure
    assert [len(x) for x in reps_b] == [1200] * n + [0] * (r - n) == [int(x) for x in rl]
    assert fps_b == [int(x) for x in fp]
    assert all(a.tobytes() == rep[i].tobytes() for i, a in enumerate(reps_b[:n]))
    bt.close()


class _WindowSc:
    """fecgpu_set_knob("window_sc", v) for a block (1: the shared-coefficient stream kernel, 0: the
    row-table fallback), through the library the mini host links."""

    def __init__(self, bt, v):
        self.L, self.v = bt.L, v

    def __enter__(self):
        self.old = C.c_int(0)
        assert self.L.fecgpu_get_knob(b"window_sc", C.byref(self.old)) == 0
        assert self.L.fecgpu_set_knob(b"window_sc", self.v) == 0

    def __exit__(self, *a):
        self.L.fecgpu_set_knob(b"window_sc", self.old.value)


@pytest.mark.parametrize("batch_blocks,window_sc", [(7, 1), (64, 1), (4096, 1), (64, 0)])
def test_batch_window_generate_sliding(batch_blocks, window_sc):
    """pquic_fec_batch_generate_window: sliding windows of several connections (window sender:
    block number 0, window_framework_sender.h:215-235), submitted interleaved in sending order, with
    steps 1-7, a gap, a repeated window, k changing mid-stream, ragged and tiny symbols and k = r = 1.
    Each window's repairs and FPIDs equal the oracle's block-number-0 encode of its symbols (zero-padded
    to the window's longest), and each connection's symbols are staged once per batch, not per window."""
    rng = np.random.default_rng(batch_blocks + window_sc)
    bt = Batch(batch_blocks, max_symbol=1500)
    o = Oracle()
    streams = []  # (symbols, [(start, k)], r)
    lens_kinds = [lambda: 1200, lambda: 1200, lambda: int(rng.integers(1, 1501)), lambda: int(rng.integers(1, 40))]
    for c in range(8):
        n = 160
        syms = [rng.integers(0, 256, lens_kinds[c % 4](), dtype=np.uint8) for _ in range(n)]
        step = [1, 2, 3, 7, 1, 5, 2, 4][c]
        k = [30, 20, 30, 12, 1, 30, 16, 25][c]
        r = [4, 4, 8, 2, 1, 6, 4, 5][c]
        wins = [(s0, k) for s0 in range(0, n - k - 40, step)]
        wins.append((wins[-1][0] + k + 3, k))  # a gap: nothing shared with the window before
        wins.append(wins[-1])                  # the same window again
        k2 = max(1, k - 3)                      # window length changes (another queue)
        wins += [(s0, k2) for s0 in range(wins[-1][0] + 1, n - k2, step)]
        streams.append((syms, wins, r))
    sids = [bt.open_stream(syms) for syms, _, _ in streams]
    pending = [list(w) for _, w, _ in streams]
    tickets = []
    now = 0
    with _WindowSc(bt, window_sc):
        while any(pending):
            for c, (syms, _, r) in enumerate(streams):
                if pending[c]:
                    s0, k = pending[c].pop(0)
                    tickets.append((c, s0, k, r, bt.generate_window(sids[c], s0, k, r, now=now)))
                    now += 1
                    if now % 97 == 0:
                        bt.L.mh_batch_poll(now)
        bt.L.mh_batch_drain()
    for c, s0, k, r, t in tickets:
        assert bt.status(t) == (0, 1)
        reps, fps = bt.repairs(t)
        want = o.rlc_encode_block(0, streams[c][0][s0: s0 + k], r)[1]
        assert [x.tobytes() for x in reps] == [x.tobytes() for x in want], (c, s0, k)
        assert fps == list(range(r))
    st = bt.stats()
    assert st["engine_errors"] == 0 and st["windows"] == len(tickets)
    total = sum(k for _, _, k, _, _ in tickets)
    if batch_blocks >= 64:  # every connection's run is staged once: rows ~ symbols, far below sum(k)
        assert st["window_rows"] < total / 3, (st["window_rows"], total)
    bt.close()


def test_batch_window_generate_fixtures():
    """Window generate on the window fixtures' RLC blocks encoded as block number 0 (window_cases.json,
    reference-generated): the repairs equal the oracle's, and fed with the fixture's erasures to the
    batched recover they give back exactly the symbols the reference recovered."""
    bt = Batch(16)
    o = Oracle()
    d = load("window_cases.json")
    jobs = []
    for i, case in enumerate(d["cases"]):
        if case["scheme"] != "rlc" or case["mixed_seeds"] or case["crashed"]:
            continue
        srcs, want, fpids = window_inputs(case, o)
        sid = bt.open_stream(srcs)
        jobs.append((case, srcs, want, fpids, bt.generate_window(sid, 0, case["k"], case["r"], now=i)))
    assert len(jobs) > 40
    bt.L.mh_batch_drain()
    rec_jobs = []
    for case, srcs, want, fpids, t in jobs:
        assert bt.status(t) == (0, 1), case["tag"]
        reps, _ = bt.repairs(t)
        assert [x.tobytes() for x in reps] == [x.tobytes() for x in want], case["tag"]
        k, r = case["k"], case["r"]
        s_in = [None if j in case["src_missing"] else srcs[j] for j in range(k)]
        r_in = [reps[x] if x in case["rep_present"] else None for x in range(r)]
        rec_jobs.append((case, bt.recover(False, case["fbn"], s_in, r_in, fpids)))
    bt.L.mh_batch_drain()
    for case, t in rec_jobs:
        ret, calls = bt.status(t)
        assert calls == 1 and ret == case["ret"], case["tag"]
        rec, _ = bt.recovered(t)
        assert {str(j): sha(v.tobytes()) for j, v in sorted(rec.items())} == case["recovered"], case["tag"]
    assert bt.stats()["windows"] == len(jobs)
    bt.close()


def test_batch_generate_arena_full_part_way_through_a_block():
    """A block whose repair symbols are split between the registered arena and other memory (the
    arena fills up part way through the block's allocations): the repairs written in place keep
    their bytes and the staged ones are copied out (advisor finding, round 3: the copy-out used to
    overwrite the in-place rows with stale staging bytes)."""
    # 13 slots: the first block's 4 sources (8 slots), repairs 0-1 (4 slots) and repair 2's struct;
    # repair 2's data and repair 3 come from the heap, as do the later blocks
    bt = Batch(4, max_symbol=1200, arena=True, arena_bytes=13 * 2112)
    rng = np.random.default_rng(11)
    o = Oracle()
    jobs = []
    for b in range(3):
        srcs = [rng.integers(0, 256, 1200, dtype=np.uint8) for _ in range(4)]
        fbn = int(rng.integers(0, 1 << 24))
        rep = o.rlc_encode_batch(np.stack(srcs)[None], 4, fbn)[0]
        jobs.append((False, fbn, srcs, 4, ("hex", [x.tobytes().hex() for x in rep]),
                     [(fbn << 8) | i for i in range(4)], 0))
    tickets = [bt.generate(*j[:4], now=i) for i, j in enumerate(jobs)]
    bt.L.mh_batch_drain()
    for t, j in zip(tickets, jobs):
        _check_generate(bt, t, j)
    st = bt.stats()
    assert st["engine_errors"] == 0
    assert st["rows_in_place"] == 4 + 2 and st["rows_staged"] > 0
    bt.close()


def _random_recover_jobs(rng, n, L, kmax=32, rmax=8):
    """RLC blocks of L-byte symbols with up to r random erasures, all repairs present, with the
    oracle's expected recovery (status, {j: bytes})."""
    o = Oracle()
    jobs = []
    for _ in range(n):
        k, r = int(rng.integers(2, kmax + 1)), int(rng.integers(1, rmax + 1))
        fbn = int(rng.integers(0, 1 << 24))
        full = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
        reps = o.rlc_encode_block(fbn, full, r)[1]
        e = int(rng.integers(1, min(k, r) + 1))
        miss = set(int(x) for x in rng.choice(k, e, replace=False))
        srcs = [None if j in miss else full[j] for j in range(k)]
        st, rec = o.rlc_decode_block(fbn, srcs, list(reps))
        jobs.append((fbn, srcs, list(reps), [(fbn << 8) | i for i in range(r)], st, rec))
    return jobs


@pytest.mark.parametrize("batch_blocks", [3, 64])
def test_batch_recover_gathers_from_connection_arenas(batch_blocks):
    """RLC recover batches read the received symbols where they lie in the connections' registered
    arenas (one per connection, as each plugin instance owns its memory) and the kernel writes each
    recovered source into the symbol allocated for it at submission.  Blocks whose length is not the
    stride, rows outside an arena and XOR blocks are staged.  Everything against the reference
    fixtures and the oracle; every symbol freed (pre-allocated symbols of unrecovered sources too)."""
    ncon = 5
    bt = Batch(batch_blocks, max_symbol=1200, connections=ncon, conn_bytes=8 << 20)
    fx = [j for j in _decode_jobs() if max([len(x) for x in j[1] + j[2] if x is not None] + [1]) <= 1200]
    rng = np.random.default_rng(batch_blocks)
    rnd = _random_recover_jobs(rng, 120, 1200)
    tickets = []
    for i, (case, srcs, reps, fp) in enumerate(fx):
        bt.use(i % ncon)
        tickets.append(bt.recover(case["scheme"] == "xor", case["fbn"], srcs, reps, fp, now=i))
    for i, (fbn, srcs, reps, fp, _, _) in enumerate(rnd):
        bt.use((i * 3) % ncon)
        tickets.append(bt.recover(False, fbn, srcs, reps, fp, now=len(fx) + i))
    bt.L.mh_batch_drain()
    for t, (case, srcs, _, _) in zip(tickets, fx):
        ret, calls = bt.status(t)
        assert calls == 1, case["tag"]
        rec, cur = bt.recovered(t)
        if case["crashed"]:
            assert ret == 0 and rec == {}
            continue
        assert ret == case["ret"], case["tag"]
        assert {str(j): sha(v.tobytes()) for j, v in sorted(rec.items())} == case["recovered"], case["tag"]
        assert {str(j): len(v) for j, v in rec.items()} == case["recovered_len"]
        present = sum(s is not None for s in srcs)
        assert cur == (present + len(rec) if case["scheme"] == "rlc" else present)
    n_rec = 0
    for t, (fbn, srcs, _, _, st, want) in zip(tickets[len(fx):], rnd):
        ret, calls = bt.status(t)
        assert calls == 1 and ret == 0
        rec, cur = bt.recovered(t)
        assert sorted(rec) == sorted(want), fbn
        for j in rec:
            assert rec[j].tobytes() == want[j].tobytes(), (fbn, j)
            assert bt.last_fpids[j] == ((fbn << 8) + j) & 0xFFFFFFFF
        assert cur == sum(s is not None for s in srcs) + len(rec)
        n_rec += len(rec)
    assert n_rec > 100
    st = bt.stats()
    assert st["engine_errors"] == 0
    assert st["rows_in_place"] > 1000, st
    bt.close()


def test_batch_many_connection_arenas():
    """More than a thousand registered arenas (one per connection): every block's rows are found in
    its connection's arena (sorted registry, binary search) and coded in place."""
    ncon = 1100
    bt = Batch(512, max_symbol=1200, connections=ncon, conn_bytes=64 << 10)
    rng = np.random.default_rng(5)
    o = Oracle()
    jobs = []
    for c in range(ncon):
        srcs = [rng.integers(0, 256, 1200, dtype=np.uint8) for _ in range(4)]
        fbn = int(rng.integers(0, 1 << 24))
        rep = o.rlc_encode_batch(np.stack(srcs)[None], 2, fbn)[0]
        jobs.append((False, fbn, srcs, 2, ("hex", [x.tobytes().hex() for x in rep]),
                     [(fbn << 8) | i for i in range(2)], 0))
    tickets = []
    for c, j in enumerate(jobs):
        bt.use(c)
        tickets.append(bt.generate(*j[:4], now=c))
    bt.L.mh_batch_drain()
    for t, j in zip(tickets, jobs):
        _check_generate(bt, t, j)
    st = bt.stats()
    assert st["engine_errors"] == 0
    assert st["rows_in_place"] == ncon * (4 + 2) and st["rows_staged"] == 0, st
    bt.close()


def test_batch_completions_follow_submission_order():
    """Blocks of one queue complete in submission order across batches, although two engine threads
    (and copy-out passes) can finish batches out of order."""
    bt = Batch(3, max_symbol=1200)
    rng = np.random.default_rng(3)
    tickets = []
    for i in range(60):
        srcs = [rng.integers(0, 256, 1200, dtype=np.uint8) for _ in range(8)]
        tickets.append(bt.generate(False, i, srcs, 4, now=i))
    bt.L.mh_batch_drain()
    order = [bt.L.mh_batch_order(t) for t in tickets]
    assert order == sorted(order) and min(order) >= 0
    bt.close()


@pytest.mark.gpu
def test_batch_connection_closes_arena_unregistered():
    """A connection closing takes its arena out of the registry (pquic_fec_batch_unregister_heap) while
    the others keep theirs: that connection's rows are staged from then on, the others' stay in place,
    every repair still equals the reference's, and the range cannot be unregistered twice."""
    ncon = 4
    bt = Batch(8, max_symbol=1200, connections=ncon, conn_bytes=256 << 10)
    bt.L.mh_batch_unregister_connection.argtypes = [C.c_int]
    rng = np.random.default_rng(11)
    o = Oracle()

    def job():
        srcs = [rng.integers(0, 256, 1200, dtype=np.uint8) for _ in range(6)]
        fbn = int(rng.integers(0, 1 << 24))
        rep = o.rlc_encode_batch(np.stack(srcs)[None], 3, fbn)[0]
        return (False, fbn, srcs, 3, ("hex", [x.tobytes().hex() for x in rep]), [(fbn << 8) | i for i in range(3)], 0)

    def run(conns):
        done = []
        for c in conns:
            bt.use(c)
            j = job()
            done.append((bt.generate(*j[:4], now=len(done)), j))
        bt.L.mh_batch_drain()
        for t, j in done:
            _check_generate(bt, t, j)

    run(list(range(ncon)) * 4)
    st0 = bt.stats()
    assert st0["rows_staged"] == 0 and st0["rows_in_place"] == 16 * (6 + 3)
    assert bt.L.mh_batch_unregister_connection(1) == 0
    assert bt.L.mh_batch_unregister_connection(1) != 0  # not registered any more
    run([0, 1, 2, 3, 1, 1])
    st1 = bt.stats()
    assert st1["rows_staged"] - st0["rows_staged"] == 3 * (6 + 3)
    assert st1["rows_in_place"] - st0["rows_in_place"] == 3 * (6 + 3)
    assert st1["engine_errors"] == 0
    bt.close()


def test_batch_recover_arena_full_part_way_through_a_block():
    """Recover on the gather path when the arena fills part way through a block's allocations: the
    first block's received symbols (12 slots) and its first recovered symbol (2 slots) lie in the
    registered arena, its second recovered symbol's data and everything after come from the heap.
    The recovered rows written in place keep their bytes, the staged ones are copied in, and every
    block equals the oracle's recovery."""
    k, r, L = 6, 3, 1200
    bt = Batch(4, max_symbol=L, arena=True, arena_bytes=15 * 2112)
    rng = np.random.default_rng(17)
    o = Oracle()
    jobs = []
    for b in range(3):
        fbn = int(rng.integers(0, 1 << 24))
        full = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
        reps = o.rlc_encode_block(fbn, full, r)[1]
        miss = {1, 3, 4}
        srcs = [None if j in miss else full[j] for j in range(k)]
        st, rec = o.rlc_decode_block(fbn, srcs, list(reps))
        assert sorted(rec) == sorted(miss)
        t = bt.recover(False, fbn, srcs, list(reps), [(fbn << 8) | i for i in range(r)], now=b)
        jobs.append((t, fbn, srcs, rec))
    bt.L.mh_batch_drain()
    for t, fbn, srcs, want in jobs:
        ret, calls = bt.status(t)
        assert calls == 1 and ret == 0
        got, cur = bt.recovered(t)
        assert sorted(got) == sorted(want), fbn
        for j in got:
            assert got[j].tobytes() == want[j].tobytes(), (fbn, j)
            assert bt.last_fpids[j] == ((fbn << 8) + j) & 0xFFFFFFFF
        assert cur == sum(s is not None for s in srcs) + len(got)
    st = bt.stats()
    assert st["engine_errors"] == 0
    assert st["rows_in_place"] == 6 + 1 and st["rows_staged"] > 0, st
    bt.close()


def test_batch_recover_frees_unrecovered_preallocations_first():
    """A gathered recover allocates a symbol for every missing source at submission; the reference
    allocates only for the sources it recovers, after decoding (rlc_fec_scheme_gf256.c:218-236).  The block:
    k8 r4, sources 2, 3, 5, 6 missing, source 6 all zero, so only source 5 is recovered (the zero rule
    drops 6 and what depends on it, :98-101).  The plugin arena returns NULL once full (my_malloc_block
    without dynamic memory, picoquic/memory.c:72-110) and has three slots left after the received symbols:
    the pre-allocations of 2, 3 and 5 fail (injected), 6's takes two slots.  The completion frees 6's
    symbol before it allocates 5's anew, so source 5 is recovered, as the reference recovers it;
    allocating in source order first would have found one free slot and skipped it."""
    k, r, L = 8, 4, 1200
    # 40960 B = 19 slots of 2112 B: 8 for the four received sources, 8 for the four repairs, 3 left
    bt = Batch(1, max_symbol=L, arena=True, arena_bytes=40960)
    bt.L.mh_arena_strict.argtypes = [C.c_int]
    bt.L.mh_fail_alloc_range.argtypes = [C.c_long, C.c_long]
    bt.L.mh_fail_alloc_after.argtypes = [C.c_long]
    rng = np.random.default_rng(4)
    o = Oracle()
    full = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    fbn = int(rng.integers(0, 1 << 24))
    full[6] = np.zeros(L, np.uint8)
    reps = o.rlc_encode_block(fbn, full, r)[1]
    miss = (2, 3, 5, 6)
    srcs = [None if j in miss else full[j] for j in range(k)]
    st, want = o.rlc_decode_block(fbn, srcs, list(reps))
    assert sorted(want) == [5]
    bt.L.mh_arena_strict(1)
    try:
        # allocations 0-15 build the received block; 16-21 are the pre-allocations of sources 2, 3, 5
        # (symbol, then data, each), 22-23 source 6's
        bt.L.mh_fail_alloc_range(2 * 4 + 2 * 4, 6)
        t = bt.recover(False, fbn, srcs, list(reps), [(fbn << 8) | i for i in range(r)])
        bt.L.mh_batch_drain()
    finally:
        bt.L.mh_fail_alloc_after(-1)
        bt.L.mh_arena_strict(0)
    ret, calls = bt.status(t)
    assert calls == 1 and ret == 0
    got, cur = bt.recovered(t)
    assert sorted(got) == [5]
    assert got[5].tobytes() == want[5].tobytes()
    assert bt.last_fpids[5] == (fbn << 8) + 5
    assert cur == k - len(miss) + 1
    bt.close()
