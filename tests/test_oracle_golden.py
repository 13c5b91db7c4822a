"""The CPU restatement (oracle/) against fixtures produced by the reference itself.

Every expected value was produced by the reference's own plugins/fec scheme pluglets
compiled natively (tests/golden/gen_golden.py); nothing here depends on a GPU.
"""
import numpy as np
import pytest

from golden_io import decode_sources, encode_inputs, load, load_npz, sha, window_inputs
from oracle_py import DEC_NOTHING, DEC_RECOVERED, DEC_REF_UB, Oracle


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


def test_gf256_tables(oracle):
    g = load("gf256_tables.json")
    mul, inv = oracle.gf_tables()
    assert inv.tobytes().hex() == g["inv_hex"]
    assert sha(mul.tobytes()) == g["mul_sha256"]
    for a, b, p in g["mul_kat"]:
        assert mul[a, b] == p
    # SURVEY.md §8a A1 known answers
    assert mul[2, 0x80] == 0x1D and mul[0x53, 0xCA] == 0x8F and mul[0xFF, 0xFF] == 0xE2
    assert inv[0x53] == 0x8C and inv[0] == 0


def test_tinymt32_streams(oracle):
    t = load("tinymt32.json")
    for seed, stream in t["streams"].items():
        got = oracle.tinymt32(int(seed), len(stream))
        assert [int(x) for x in got] == stream, seed
    assert int(oracle.tinymt32(1, 1)[0]) == 0x97B6D625  # published TinyMT32 check value


def test_coefficient_kat(oracle):
    # SURVEY.md Appendix A
    assert oracle.coefs(0x700, 16).tobytes().hex() == "aa6e58dca8a888451b77e9536767571f"
    assert oracle.coefs(0x701, 16).tobytes().hex() == "2f78cf7da35d9f9dc75557285c0d3161"
    assert oracle.coefs(0, 16).tobytes().hex() == "272a99d0b0db4d4885a326acba7f8aec"
    assert oracle.coefs(0x12345605, 16).tobytes().hex() == "7a929bb13425c197ff4a8ce2d9c428ed"
    assert oracle.seed(0x123456, 5) == 0x12345605
    assert oracle.seed(0x1234567, 5) == 0x23456705  # fec_block_number is a 24-bit field
    c = oracle.coefs(0, 4096)
    assert (c != 0).all()


def test_deterministic_encode_kat(oracle):
    # S_j[t] = (j*31 + t*7 + 1) & 0xff, fbn 7
    expect = {(16, 4, 1200): "b73a4ef60eeb2373836877dfaf9ccc82f810ab9ad4fc435c184b4f5fcd91690e",
              (32, 8, 1200): "b98d6d841a89de7a5fa7839d849d89619035875ce033a6f9ca1f2b83971e7708"}
    for (k, r, L), h in expect.items():
        srcs = [np.array([(j * 31 + t * 7 + 1) & 0xFF for t in range(L)], np.uint8) for j in range(k)]
        ret, reps = oracle.rlc_encode_block(7, srcs, r)
        assert ret == 0 and sha(b"".join(x.tobytes() for x in reps)) == h
    srcs = [np.array([(j * 31 + t * 7 + 1) & 0xFF for t in range(1200)], np.uint8) for j in range(4)]
    ret, rep = oracle.xor_encode_block(srcs)
    assert sha(rep.tobytes()) == "c1bf9684ffb00fc43147e70159eabbbe0f0f20cb3a6291111609285d342112b8"


def test_encode_cases(oracle):
    e = load("encode_cases.json")
    full = load_npz("encode_full.npz")
    for case in e["cases"]:
        src = encode_inputs(case)
        if case["scheme"] == "xor":
            rep = oracle.xor_encode_batch(src)
        else:
            rep = oracle.rlc_encode_batch(src, case["r"], case["fbn_base"])
        assert [sha(rep[b].tobytes()) for b in range(case["nblocks"])] == case["block_sha256"], case["name"]
        if "enc_" + case["name"] in full:
            assert np.array_equal(rep, full["enc_" + case["name"]])


def test_encode_varlen_and_preconditions(oracle):
    e = load("encode_cases.json")
    for case in e["varlen"]:
        srcs = [np.frombuffer(bytes.fromhex(h), np.uint8) for h in case["src_hex"]]
        if case["scheme"] == "xor":
            ret, rep = oracle.xor_encode_block(srcs)
            reps = [rep]
        else:
            ret, reps = oracle.rlc_encode_block(case["fbn"], srcs, case["r"])
        assert ret == case["ret"]
        assert [x.tobytes().hex() for x in reps] == case["rep_hex"]
    for p in e["preconditions"]:
        srcs = [np.arange(10, dtype=np.uint8) + j for j in range(p["k"])]
        if p["scheme"] == "xor":
            got = 1 if p["r"] != 1 else oracle.xor_encode_block(srcs)[0]
        else:
            got = oracle.rlc_encode_block(3, srcs, p["r"])[0]
        assert got == p["ret"]


def _check_decode(oracle, case):
    srcs_full = decode_sources(case)
    k, r = case["k"], case["r"]
    fbn = case["fbn"]
    if case["scheme"] == "xor":
        _, rep = oracle.xor_encode_block(srcs_full)
        reps_full = [rep]
    else:
        _, reps_full = oracle.rlc_encode_block(fbn, srcs_full, r)
    srcs = [None if j in case["src_missing"] else srcs_full[j] for j in range(k)]
    reps = [reps_full[i] if i in case["rep_present"] else None for i in range(r)]
    if case["scheme"] == "xor":
        st, rec = oracle.xor_decode_block(srcs, reps)
    else:
        st, rec = oracle.rlc_decode_block(fbn, srcs, reps)
    if case["crashed"]:
        assert st == DEC_REF_UB, case["tag"]
        return st
    assert st != DEC_REF_UB, case["tag"]
    if case["scheme"] == "xor":
        assert (st == DEC_RECOVERED) == (case["ret"] == 0), case["tag"]
    else:
        assert case["ret"] == 0
    got = {str(j): sha(v.tobytes()) for j, v in sorted(rec.items())}
    assert got == case["recovered"], case["tag"]
    assert {str(j): len(v) for j, v in rec.items()} == case["recovered_len"]
    return st


def test_decode_cases(oracle):
    d = load("decode_cases.json")
    seen = set()
    for case in d["cases"]:
        seen.add(_check_decode(oracle, case))
    assert {DEC_RECOVERED, DEC_NOTHING, DEC_REF_UB} <= seen


def test_decode_zero_symbols(oracle):
    d = load("decode_cases.json")
    partial = 0
    for case in d["zero_cases"]:
        _check_decode(oracle, case)
        partial += 0 < len(case["recovered"]) < len(case["src_missing"])
    assert partial > 0  # the fixture set exercises dependency propagation


def test_decode_varlen(oracle):
    d = load("decode_cases.json")
    for case in d["varlen_cases"]:
        _check_decode(oracle, case)


def test_decode_batch_roundtrip(oracle):
    """Batched driver: encode -> erase e sources -> decode restores the originals."""
    rng = np.random.default_rng(3)
    nb, k, r, L = 64, 16, 4, 1200
    from oracle_py import synth_bytes
    src = synth_bytes(nb * k * L, 77).reshape(nb, k, L)
    rep = oracle.rlc_encode_batch(src, r, 10)
    sp = np.zeros((nb, 2), np.uint64)
    rp = np.zeros((nb, 2), np.uint64)
    work = src.copy()
    for b in range(nb):
        miss = rng.choice(k, size=4, replace=False)
        m = (1 << k) - 1
        for j in miss:
            m &= ~(1 << int(j))
            work[b, j] = 0xA5
        sp[b, 0] = m
        rp[b, 0] = (1 << r) - 1
    st, rec = oracle.rlc_decode_batch(work, rep, sp, rp, 10)
    ok = st == DEC_RECOVERED
    assert ok.sum() > nb * 0.9
    assert np.array_equal(work[ok], src[ok])
    assert ((st == DEC_RECOVERED) | (st == DEC_REF_UB)).all()


def test_decode_window_framework_blocks(oracle):
    """Window-framework-shaped blocks (window_cases.json): the block is numbered by its window
    start, the repairs carry block number 0 (or mixed block numbers) and every equation is seeded
    by its repair's own FPID (rlc_fec_scheme_gf256.c:200)."""
    d = load("window_cases.json")
    seen = set()
    for case in d["cases"]:
        srcs_full, reps_full, fpids = window_inputs(case, oracle)
        k, r = case["k"], case["r"]
        srcs = [None if j in case["src_missing"] else srcs_full[j] for j in range(k)]
        reps = [reps_full[i] if i in case["rep_present"] else None for i in range(r)]
        if case["scheme"] == "xor":
            st, rec = oracle.xor_decode_block(srcs, reps)
        else:
            st, rec = oracle.rlc_decode_block(case["fbn"], srcs, reps, [f & 0xFFFFFFFF for f in fpids])
        seen.add(st)
        if case["crashed"]:
            assert st == DEC_REF_UB, case["tag"]
            continue
        assert st != DEC_REF_UB, case["tag"]
        assert {str(j): sha(v.tobytes()) for j, v in sorted(rec.items())} == case["recovered"], case["tag"]
        assert {str(j): len(v) for j, v in rec.items()} == case["recovered_len"], case["tag"]
        fb = case["fbn"]
        assert {str(j): ((fb << 8) + j) & 0xFFFFFFFF for j in rec} == case["recovered_fpid"], case["tag"]
    assert DEC_RECOVERED in seen and DEC_REF_UB in seen
    assert any(c["mixed_seeds"] and c["recovered"] for c in d["cases"])
    # block-number seeds instead of the FPIDs would NOT reproduce the reference: the gap the
    # adapter closes (seeding by (window start << 8) | i recovers wrong bytes)
    case = next(c for c in d["cases"] if c["scheme"] == "rlc" and c["recovered"] and not c["crashed"])
    srcs_full, reps_full, _ = window_inputs(case, oracle)
    srcs = [None if j in case["src_missing"] else srcs_full[j] for j in range(case["k"])]
    reps = [reps_full[i] if i in case["rep_present"] else None for i in range(case["r"])]
    _, wrong = oracle.rlc_decode_block(case["fbn"], srcs, reps)
    assert {str(j): sha(v.tobytes()) for j, v in sorted(wrong.items())} != case["recovered"]
