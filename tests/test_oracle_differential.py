"""The CPU oracle (oracle/fec_oracle.c) against the reference's scheme pluglets, live, on random blocks
beyond the committed fixtures: random k, r, L (fixed or variable symbol lengths), block numbers,
erasure patterns, repair subsets and all-zero sources, encode and decode, RLC and XOR.  The reference
is the native build in oracle/_ref (`make -C oracle ref`; its decode runs in a fork()ed child, so the
patterns that crash it are observed: the oracle must report DEC_REF_UB for exactly those).  Skips
where that build is absent (the GPU boxes).  CPU suite; together with tests/test_oracle_golden.py this
pins the oracle that the GPU parity tests check the engine against."""
import faulthandler
import os
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from oracle_py import DEC_RECOVERED, DEC_REF_UB, REF_PATH, Oracle, Reference  # noqa: E402

N = int(os.environ.get("PQUIC_ORACLE_FUZZ_CASES", "300"))


@pytest.fixture(scope="module")
def pair():
    if not os.path.exists(REF_PATH):
        pytest.skip("reference build oracle/_ref/libfecref.so absent")
    return Oracle(), Reference()


def _block(rng):
    k = int(rng.choice([1, 2, 4, 5, 8, 16, 25, 32, 64, int(rng.integers(1, 65))]))
    r = int(rng.choice([1, 2, 3, 4, 8, 16, int(rng.integers(1, 17))]))
    L = int(rng.choice([1, 8, 40, 100, 1200, int(rng.integers(1, 1500))]))
    if rng.random() < 0.25:  # variable lengths (the encode pads to the longest, rlc_fec_scheme_generate_gf256.c:41-55)
        srcs = [rng.integers(0, 256, int(rng.integers(1, L + 1)), dtype=np.uint8) for _ in range(k)]
    else:
        srcs = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    if rng.random() < 0.15:  # all-zero sources: dropped with what depends on them (rlc_fec_scheme_gf256.c:98-101)
        for j in rng.choice(k, size=int(rng.integers(1, min(k, 3) + 1)), replace=False):
            srcs[j] = np.zeros(len(srcs[j]), np.uint8)
    return k, r, srcs, int(rng.integers(0, 1 << 24))


def test_encode_differential(pair):
    oracle, ref = pair
    rng = np.random.default_rng(8101)
    for t in range(N):
        k, r, srcs, fbn = _block(rng)
        ret, reps, _ = ref.encode_block(False, fbn, srcs, r)
        oret, oreps = oracle.rlc_encode_block(fbn, srcs, r)
        assert oret == ret, (t, k, r)
        if ret == 0:
            assert len(oreps) == len(reps) and all(np.array_equal(a, b) for a, b in zip(oreps, reps)), (t, k, r)
        xret, xreps, _ = ref.encode_block(True, fbn, srcs, 1)
        oxret, oxrep = oracle.xor_encode_block(srcs)
        assert oxret == xret, (t, k)
        if xret == 0:
            assert np.array_equal(oxrep, xreps[0]), (t, k)


@pytest.fixture
def quiet_crashes():
    """the reference's crashes happen in fork()ed children, which inherit pytest's faulthandler: keep
    their tracebacks out of the log while the decodes run"""
    was = faulthandler.is_enabled()
    faulthandler.disable()
    yield
    if was:
        faulthandler.enable()


def test_decode_differential(pair, quiet_crashes):
    oracle, ref = pair
    rng = np.random.default_rng(8102)
    crashed = recovered = 0
    for t in range(N):
        k, r, srcs_full, fbn = _block(rng)
        xor = r == 1 and rng.random() < 0.5
        ret, reps_full, fpids = ref.encode_block(xor, fbn, srcs_full, r)
        assert ret == 0
        e = int(rng.integers(1, min(k, r + 1) + 1))
        missing = set(int(j) for j in rng.choice(k, size=e, replace=False))
        mode = t % 3
        if mode == 0:
            present = set(range(min(e, r)))
        elif mode == 1:
            present = set(int(i) for i in rng.choice(r, size=int(rng.integers(min(e, r), r + 1)), replace=False))
        else:
            present = set(int(i) for i in rng.choice(r, size=int(rng.integers(0, r + 1)), replace=False))
        srcs = [None if j in missing else srcs_full[j] for j in range(k)]
        reps = [reps_full[i] if i in present else None for i in range(r)]
        rret, rrec = ref.decode_block(xor, fbn, srcs, reps, fpids)
        if xor:
            st, orec = oracle.xor_decode_block(srcs, reps)
        else:
            st, orec = oracle.rlc_decode_block(fbn, srcs, reps)
        tag = (t, "xor" if xor else "rlc", k, r, sorted(missing), sorted(present))
        if rret <= -1000:  # the reference crashed on this pattern
            crashed += 1
            assert st == DEC_REF_UB, tag
            continue
        assert st != DEC_REF_UB, tag
        if xor:
            assert (st == DEC_RECOVERED) == (rret == 0), tag
        assert sorted(orec) == sorted(rrec), tag
        assert all(np.array_equal(orec[j], rrec[j]) for j in rrec), tag
        recovered += len(rrec)
    assert recovered > N  # most cases recover something; crashes are allowed, not required
