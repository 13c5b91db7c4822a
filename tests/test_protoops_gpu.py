"""The drop-in protocol operations (include/pquic_fec_protoops.h), driven through a minimal
picoquic stand-in (tests/host/mini_host.c) exactly as the block framework calls the
reference pluglets, against fixtures produced by the reference pluglets themselves."""
import ctypes as C
import os

import numpy as np
import pytest

from golden_io import decode_sources, load, sha, window_inputs
from oracle_py import Oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
# PQUIC_TEST_MINIHOST: a sanitizer build over the CPU engine stand-in (tests/sanitize, test_sanitize.py)
MINIHOST = os.environ.get("PQUIC_TEST_MINIHOST") or os.path.join(ROOT, "tests", "host", "libminihost.so")


def _p(a, t=C.c_uint8):
    return a.ctypes.data_as(C.POINTER(t))


class Host:
    def __init__(self):
        self.lib = C.CDLL(MINIHOST)
        self.lib.mh_generate.restype = C.c_long
        self.lib.mh_recover.restype = C.c_long
        self.lib.mh_live_allocations.restype = C.c_long
        assert self.lib.mh_bind(0) == 0

    def generate(self, xor, fbn, srcs, r):
        k = len(srcs)
        stride = max([len(s) for s in srcs] + [1])
        buf = np.zeros((k, stride), np.uint8)
        lens = np.zeros(k, np.uint16)
        for j, s in enumerate(srcs):
            buf[j, : len(s)] = s
            lens[j] = len(s)
        rep = np.zeros((max(r, 1), stride), np.uint8)
        rl = np.zeros(max(r, 1), np.uint16)
        fp = np.zeros(max(r, 1), np.uint64)
        sch = np.zeros(2, np.uint64)
        ret = self.lib.mh_generate(int(xor), fbn, k, r, _p(buf), _p(lens, C.c_uint16), stride, _p(rep),
                                   _p(rl, C.c_uint16), _p(fp, C.c_uint64), stride, _p(sch, C.c_uint64))
        return ret, [rep[i, : rl[i]].copy() for i in range(r)], [int(x) for x in fp[:r]], sch

    def recover(self, xor, fbn, srcs, reps, fpids):
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
        out = np.zeros((k, stride), np.uint8)
        ol = np.zeros(k, np.uint16)
        rec = np.zeros(k, np.uint8)
        cur = C.c_int(0)
        ofp = np.zeros(k, np.uint32)
        ret = self.lib.mh_recover(int(xor), fbn, k, r, _p(sb), _p(sl, C.c_uint16), _p(spres), stride, _p(rb),
                                  _p(rl, C.c_uint16), _p(rpres), _p(fp, C.c_uint64), stride, _p(out),
                                  _p(ol, C.c_uint16), _p(rec), stride, C.byref(cur), _p(ofp, C.c_uint32))
        self.last_fpids = {j: int(ofp[j]) for j in range(k) if rec[j]}
        return ret, {j: out[j, : ol[j]].copy() for j in range(k) if rec[j]}, cur.value


@pytest.fixture(scope="module")
def host():
    return Host()


def test_generate_varlen_matches_reference(host):
    e = load("encode_cases.json")
    for case in e["varlen"]:
        srcs = [np.frombuffer(bytes.fromhex(h), np.uint8) for h in case["src_hex"]]
        ret, reps, fps, sch = host.generate(case["scheme"] == "xor", case["fbn"], srcs, case["r"])
        assert ret == case["ret"]
        assert [x.tobytes().hex() for x in reps] == case["rep_hex"]
        assert fps == case["repair_fpid_raw"]
        if case["scheme"] == "rlc":
            assert sch[0] == sch[1] != 0   # one scheme object for both directions
        else:
            assert sch[0] == sch[1] == 0   # create_xor_fec_scheme.c:6-7


def test_generate_fixed_cases_and_preconditions(host):
    from golden_io import encode_inputs, load_npz
    e = load("encode_cases.json")
    full = load_npz("encode_full.npz")
    for case in e["cases"]:
        if case["k"] > 100 or case["r"] > 100:
            continue
        src = encode_inputs(case)
        for b in range(case["nblocks"]):
            fbn = (case["fbn_base"] + b) & 0xFFFFFF
            ret, reps, fps, _ = host.generate(case["scheme"] == "xor", fbn, list(src[b]), case["r"])
            assert ret == 0
            assert sha(np.stack(reps).tobytes()) == case["block_sha256"][b], case["name"]
            assert fps == case["repair_fpid_raw"][b]
    for p in e["preconditions"]:
        srcs = [np.arange(10, dtype=np.uint8) + j for j in range(p["k"])]
        ret, _, _, _ = host.generate(p["scheme"] == "xor", 3, srcs, p["r"])
        assert ret == p["ret"]


def _decode_case(host, case):
    srcs_full = decode_sources(case)
    k, r, fbn = case["k"], case["r"], case["fbn"]
    o = Oracle()
    if case["scheme"] == "xor":
        reps_full = [o.xor_encode_block(srcs_full)[1]]
        fpids = [fbn << 8]
    else:
        reps_full = o.rlc_encode_block(fbn, srcs_full, r)[1]
        fpids = [(fbn << 8) | i for i in range(r)]
    srcs = [None if j in case["src_missing"] else srcs_full[j] for j in range(k)]
    reps = [reps_full[i] if i in case["rep_present"] else None for i in range(r)]
    return host.recover(case["scheme"] == "xor", fbn, srcs, reps, fpids), srcs


def test_recover_matches_reference(host):
    d = load("decode_cases.json")
    n = 0
    for case in d["cases"] + d["zero_cases"] + d["varlen_cases"]:
        if case["crashed"] or case["k"] > 100:
            continue
        (ret, rec, cur), srcs = _decode_case(host, case)
        assert ret == case["ret"], case["tag"]
        got = {str(j): sha(v.tobytes()) for j, v in sorted(rec.items())}
        assert got == case["recovered"], case["tag"]
        assert {str(j): len(v) for j, v in rec.items()} == case["recovered_len"]
        present = sum(s is not None for s in srcs)
        if case["scheme"] == "rlc":
            assert cur == present + len(rec)   # rlc_fec_scheme_gf256.c:230
        else:
            assert cur == present              # xor_fec_scheme.c:72 does not count it
        n += 1
    assert n > 350


def test_recover_reference_crash_patterns_do_not_crash(host):
    d = load("decode_cases.json")
    crashed = [c for c in d["cases"] if c["crashed"]]
    assert crashed
    for case in crashed:
        (ret, rec, _), _ = _decode_case(host, case)
        assert ret == 0 and rec == {}


def test_no_leaks(host):
    base = host.lib.mh_live_allocations()
    d = load("decode_cases.json")
    for case in d["cases"][:40]:
        _decode_case(host, case)
    assert host.lib.mh_live_allocations() == base


def test_recover_window_framework_blocks(host):
    """Sliding-window framework (every shipped FEC manifest: fec.plugin:5-8,
    fec_rlc_gf256_window.plugin:5-8): the receiver numbers the block by the window start and
    slots repairs whose FPIDs carry block number 0 (window_framework_receiver.h:60-86,
    window_framework_sender.h:239-243).  fec_recover seeds each equation with the repair's own
    FPID (rlc_fec_scheme_gf256.c:200) and stamps recovered sources (start << 8) + j (:222).
    Checked against window_cases.json, produced by the reference's fec_recover."""
    o = Oracle()
    d = load("window_cases.json")
    n = 0
    for case in d["cases"]:
        srcs_full, reps_full, fpids = window_inputs(case, o)
        k, r = case["k"], case["r"]
        srcs = [None if j in case["src_missing"] else srcs_full[j] for j in range(k)]
        reps = [reps_full[i] if i in case["rep_present"] else None for i in range(r)]
        ret, rec, cur = host.recover(case["scheme"] == "xor", case["fbn"], srcs, reps, fpids)
        if case["crashed"]:  # the reference segfaults on this pattern; the adapter recovers nothing
            assert ret == 0 and rec == {}, case["tag"]
            continue
        assert ret == case["ret"], case["tag"]
        assert {str(j): sha(v.tobytes()) for j, v in sorted(rec.items())} == case["recovered"], case["tag"]
        assert {str(j): len(v) for j, v in rec.items()} == case["recovered_len"], case["tag"]
        assert {str(j): f for j, f in host.last_fpids.items()} == case["recovered_fpid"], case["tag"]
        present = sum(s is not None for s in srcs)
        assert cur == (present + len(rec) if case["scheme"] == "rlc" else present)
        n += int(bool(rec))
    assert n > 140


def test_oversized_block_rejected_before_the_device(host):
    """total_source_symbols / total_repair_symbols above the block's 100 slots (u8 fields a peer
    sets, block_framework_receiver.h:44-45): the adapter refuses the block instead of reading past
    fec_block_t as the reference would; no device call is made (the call counters do not move)."""
    st0 = np.zeros(5, np.uint64)
    host.lib.mh_protoop_stats(_p(st0, C.c_uint64))
    host.lib.mh_oversized.restype = C.c_long
    for xor, op, kt, rt in [(0, 0, 150, 4), (0, 0, 16, 120), (0, 1, 150, 20), (0, 1, 100, 101), (1, 1, 150, 1),
                            (1, 0, 150, 1)]:
        assert host.lib.mh_oversized(xor, op, kt, rt) == 0x41B
    st1 = np.zeros(5, np.uint64)
    host.lib.mh_protoop_stats(_p(st1, C.c_uint64))
    assert st1[0] == st0[0] and st1[1] == st0[1]   # no generate / recover reached the engine
    assert st1[4] == st0[4] + 6                     # six errors counted


def test_random_blocks_match_oracle(host):
    """The protocol operations on 150 random blocks beyond the fixtures, both directions, against the
    oracle (itself pinned to the reference, test_oracle_golden.py / test_oracle_differential.py).
    - Shapes: k 1-100, r 1-32, equal or variable symbol lengths, all-zero sources.
    - Inputs: random block numbers, erasures and repair subsets, RLC and XOR.
    - Patterns that crash the reference (the oracle's DEC_REF_UB) must recover nothing and return 0.
    Under the sanitizer builds (test_sanitize.py) this drives the adapters' bounds on random shapes."""
    from oracle_py import DEC_RECOVERED, DEC_REF_UB
    o = Oracle()
    rng = np.random.default_rng(0xB10C)
    for t in range(150):
        k = int(rng.choice([1, 2, 4, 5, 16, 32, 64, 100, int(rng.integers(1, 101))]))
        xor = rng.random() < 0.2
        r = 1 if xor else int(rng.choice([1, 2, 4, 8, 16, int(rng.integers(1, 33))]))
        L = int(rng.choice([1, 8, 40, 1200, int(rng.integers(1, 1500))]))
        if rng.random() < 0.3:
            srcs_full = [rng.integers(0, 256, int(rng.integers(1, L + 1)), dtype=np.uint8) for _ in range(k)]
        else:
            srcs_full = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
        if rng.random() < 0.15:
            for j in rng.choice(k, size=int(rng.integers(1, min(k, 3) + 1)), replace=False):
                srcs_full[j] = np.zeros(len(srcs_full[j]), np.uint8)
        fbn = int(rng.integers(0, 1 << 24))
        tag = (t, "xor" if xor else "rlc", k, r, L)
        ret, reps, fps, _ = host.generate(xor, fbn, srcs_full, r)
        assert ret == 0, tag
        if xor:
            want = [o.xor_encode_block(srcs_full)[1]]
        else:
            want = o.rlc_encode_block(fbn, srcs_full, r)[1]
        assert [x.tobytes() for x in reps] == [x.tobytes() for x in want], tag
        assert fps == [(fbn << 8) | i for i in range(r)], tag
        e = int(rng.integers(1, min(k, r + 1) + 1))
        missing = set(rng.choice(k, size=e, replace=False).tolist())
        present = set(rng.choice(r, size=int(rng.integers(max(0, e - 1), r + 1)), replace=False).tolist())
        srcs = [None if j in missing else srcs_full[j] for j in range(k)]
        reps_in = [reps[i] if i in present else None for i in range(r)]
        ret, rec, cur = host.recover(xor, fbn, srcs, reps_in, fps)
        if xor:
            st, orec = o.xor_decode_block(srcs, reps_in)
        else:
            st, orec = o.rlc_decode_block(fbn, srcs, reps_in)
        if st == DEC_REF_UB:
            assert ret == 0 and rec == {}, tag
            continue
        if xor:  # xor_fec_scheme.c returns non-zero when it recovers nothing; it leaves the count alone (:72)
            assert (ret == 0) == (st == DEC_RECOVERED) and cur == k - e, tag
        else:    # the RLC scheme returns 0 and counts what it inserts (rlc_fec_scheme_gf256.c:230)
            assert ret == 0 and cur == k - e + len(rec), tag
        assert sorted(rec) == sorted(orec) and all(np.array_equal(rec[j], orec[j]) for j in orec), tag
