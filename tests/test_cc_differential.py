"""Recovered packets -> congestion control against the reference pluglets, live, on random scripted
transports beyond tests/golden/cc_cases.json: the generator of tests/golden/gen_cc.py with another seed
and ten times the cases, each run through the reference (oracle/_ref/libfecref.so ref_cc_scenario /
ref_process_recovered: maybe_notify_recovered_packets_to_cc.c and process_simple_recovered_frame.c
compiled natively) and the product over the mini host (tests/host/mini_host.c mh_cc_scenario /
mh_process_recovered).  Transport-call logs, ring state and the latest notification time must match.
Skips where the reference build is absent.  CPU suite."""
import ctypes as C
import os

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
REF = os.path.join(ROOT, "oracle", "_ref", "libfecref.so")
MINIHOST = os.environ.get("PQUIC_TEST_MINIHOST") or os.path.join(ROOT, "tests", "host", "libminihost.so")
u64p, u32p, u8p = C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.POINTER(C.c_uint8)
NBUF = 50
N = int(os.environ.get("PQUIC_CC_FUZZ_CASES", "3000"))


def _bind(lib, prefix):
    sc = getattr(lib, f"{prefix}_cc_scenario")
    sc.argtypes = [C.c_int, u64p, u8p, u8p, C.c_uint64, C.c_uint64, C.c_uint64, u32p, u32p, u64p, u64p, C.c_int,
                   u64p]
    pr = getattr(lib, f"{prefix}_process_recovered")
    pr.argtypes = [u64p, C.c_int, u32p, u32p, u64p]
    return sc, pr


@pytest.fixture(scope="module")
def pair():
    if not os.path.exists(REF):
        pytest.skip("reference build oracle/_ref/libfecref.so absent")
    if not os.path.exists(MINIHOST):
        pytest.skip("mini host not built")
    return _bind(C.CDLL(REF), "ref"), _bind(C.CDLL(MINIHOST), "mh")


def _run(sc, n, pns, pure, needed, srtt, latest, now, start, size, buf):
    bs, bz = C.c_uint32(start), C.c_uint32(size)
    bout = buf.copy()
    ev = np.zeros((256, 4), np.uint64)
    lat = C.c_uint64(0)
    nev = sc(n, pns.ctypes.data_as(u64p), pure.ctypes.data_as(u8p), needed.ctypes.data_as(u8p), srtt, latest, now,
             C.byref(bs), C.byref(bz), bout.ctypes.data_as(u64p), ev.ctypes.data_as(u64p), 256, C.byref(lat))
    return nev, ev[:max(nev, 0)].tolist(), bs.value, bz.value, bout.tolist(), lat.value


def test_notify_differential(pair):
    (rsc, _), (msc, _) = pair
    rng = np.random.default_rng(9753)
    kinds = set()
    for t in range(N):
        n = int(rng.integers(0, 20))
        pns = np.cumsum(rng.integers(1, 4, n)).astype(np.uint64) + np.uint64(int(rng.integers(0, 1 << 40)))
        pure = (rng.random(n) < 0.2).astype(np.uint8)
        needed = (rng.random(n) < (0.9 if t % 4 else 0.5)).astype(np.uint8)
        cand = sorted(set(int(x) for x in list(pns) + [p - 1 for p in pns] + ([pns[-1] + 5] if n else [7])))
        m = int(rng.integers(0, min(len(cand), NBUF) + 1))
        rec = sorted(rng.choice(cand, m, replace=False).tolist()) if m else []
        if t % 7 == 3:
            rec = rec[::-1]
        start = int(rng.integers(0, NBUF))
        buf = np.zeros(NBUF, np.uint64)
        for i, p in enumerate(rec):
            buf[(start + i) % NBUF] = p
        srtt = int(rng.integers(1, 100000))
        latest = int(rng.integers(0, 1 << 30))
        now = latest + int(rng.integers(0, 2 * srtt)) if t % 5 else latest + srtt
        args = (n, pns, pure, needed, srtt, latest, now, start, len(rec), buf)
        want = _run(rsc, *args)
        assert want[0] <= 256
        assert _run(msc, *args) == want, t
        kinds |= {e[0] for e in want[1]}
    assert kinds == {1, 2, 3, 4, 5}


def test_enqueue_differential(pair):
    (_, rpr), (_, mpr) = pair
    rng = np.random.default_rng(9754)
    for t in range(N):
        start, size = int(rng.integers(0, NBUF)), int(rng.integers(0, NBUF + 1))
        buf = rng.integers(0, 1 << 50, NBUF).astype(np.uint64)
        pns = rng.integers(0, 1 << 50, int(rng.integers(0, 61))).astype(np.uint64)
        out = []
        for pr in (rpr, mpr):
            bs, bz = C.c_uint32(start), C.c_uint32(size)
            b = buf.copy()
            pr(pns.ctypes.data_as(u64p), len(pns), C.byref(bs), C.byref(bz), b.ctypes.data_as(u64p))
            out.append((bs.value, bz.value, b.tolist()))
        assert out[1] == out[0], t
