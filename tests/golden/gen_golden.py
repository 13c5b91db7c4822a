"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Runs only in the survey container, where oracle/_ref/libfecref.so is built from the
reference's own plugins/fec/fec_scheme_protoops/*.c (`make -C oracle ref`).  Every
expected value below is produced by calling those compiled reference pluglets through
get_cnx/set_cnx exactly as picoquic's protoop dispatcher would; inputs are synthetic
(oracle_py.synth_bytes) and only their seeds are stored, except where a case needs
hand-made bytes (zero symbols, variable lengths), which are stored verbatim.

    python tests/golden/gen_golden.py      # rewrites tests/golden/*.json|*.npz
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from oracle_py import Reference, synth_bytes  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def block_sources(seed: int, k: int, L: int, lens=None):
    data = synth_bytes(k * L, seed).reshape(k, L)
    if lens is None:
        return [data[j].copy() for j in range(k)]
    return [data[j, : lens[j]].copy() for j in range(k)]


def main():
    R = Reference()
    # ---- 1. GF(2^8) tables, layout, TinyMT32 -------------------------------------------
    mul, inv = R.gf_tables()
    gf = {
        "source": "create_rlc_fec_scheme_gf256.c:46-59 (assign_mul / assign_inv)",
        "inv_hex": inv.tobytes().hex(),
        "mul_sha256": sha(mul.tobytes()),
        "mul_kat": [[2, 0x80, int(mul[2, 0x80])], [0x53, 0xCA, int(mul[0x53, 0xCA])],
                    [0xFF, 0xFF, int(mul[0xFF, 0xFF])], [0x1D, 0x02, int(mul[0x1D, 0x02])]],
    }
    lay = R.layout()
    layout = {"source": "plugins/fec/fec.h:44-130 compiled with gcc x86-64",
              "sizeof_fec_block_t": lay[0], "sizeof_source_symbol_t": lay[1],
              "sizeof_repair_symbol_t": lay[2], "off_source_symbols": lay[3],
              "off_repair_symbols": lay[4], "off_source_data": lay[5], "off_repair_data": lay[6],
              "sizeof_repair_fpid_t": lay[7]}
    seeds = [0, 1, 2, 0x700, 0x701, 0x707, 0x12345605, 0xFFFFFF0F, 0xFFFFFFFF, 0x80000000]
    tmt = {"source": "prng/tinymt32.c:158-161,301-315 with mat1/mat2/tmat of "
                     "rlc_fec_scheme_generate_gf256.c:27-29",
           "streams": {str(s): [int(x) for x in R.tinymt32(s, 96)] for s in seeds}}
    with open(os.path.join(OUT, "gf256_tables.json"), "w") as f:
        json.dump(gf, f, indent=1)
    with open(os.path.join(OUT, "layout.json"), "w") as f:
        json.dump(layout, f, indent=1)
    with open(os.path.join(OUT, "tinymt32.json"), "w") as f:
        json.dump(tmt, f)

    # ---- 2. Encode vectors --------------------------------------------------------------
    enc_cases = []
    arrays = {}
    spec = [
        # (name, xor, k, r, L, nblocks, fbn_base, data_seed, keep_full)
        ("xor_k4_L1200", True, 4, 1, 1200, 6, 0, 11, True),
        ("rlc_k4_r1_L1200", False, 4, 1, 1200, 4, 0, 12, True),
        ("rlc_k16_r4_L1200", False, 16, 4, 1200, 6, 0, 13, True),
        ("rlc_k32_r8_L1200", False, 32, 8, 1200, 3, 5, 14, True),
        ("rlc_k16_r4_L1200_fbnwrap", False, 16, 4, 1200, 4, 0xFFFFFE, 15, True),
        ("rlc_k64_r16_L9000", False, 64, 16, 9000, 1, 100, 16, False),
        ("rlc_k5_r1_L64", False, 5, 1, 64, 8, 0, 17, True),
        ("rlc_k25_r5_L1200", False, 25, 5, 1200, 2, 3, 18, True),
        ("rlc_k1_r3_L16", False, 1, 3, 16, 3, 0, 19, True),
        ("rlc_k100_r100_L8", False, 100, 100, 8, 1, 9, 20, True),
    ]
    for name, xor, k, r, L, nb, fbn0, dseed, full in spec:
        src = synth_bytes(nb * k * L, dseed).reshape(nb, k, L)
        reps = np.zeros((nb, r, L), np.uint8)
        digests = []
        fpids = []
        for b in range(nb):
            fbn = (fbn0 + b) & 0xFFFFFF
            ret, rs, fp = R.encode_block(xor, fbn, [src[b, j] for j in range(k)], r)
            assert ret == 0, name
            for i in range(r):
                reps[b, i] = rs[i]
            digests.append(sha(reps[b].tobytes()))
            fpids.append(fp)
        case = {"name": name, "scheme": "xor" if xor else "rlc", "k": k, "r": r, "L": L,
                "nblocks": nb, "fbn_base": fbn0, "data_seed": dseed,
                "block_sha256": digests, "repair_fpid_raw": fpids}
        if full:
            arrays["enc_" + name] = reps
        enc_cases.append(case)

    # variable-length sources (zero padding to max length, rlc_fec_scheme_generate_gf256.c:41-55)
    var_cases = []
    rng = np.random.default_rng(1234)
    for t in range(12):
        xor = t % 3 == 0
        k = int(rng.integers(1, 9))
        r = 1 if xor else int(rng.integers(1, 5))
        lens = [int(x) for x in rng.integers(1, 1400, k)]
        srcs = [rng.integers(0, 256, n, dtype=np.uint8) for n in lens]
        fbn = int(rng.integers(0, 1 << 24))
        ret, rs, fp = R.encode_block(xor, fbn, srcs, r)
        var_cases.append({"scheme": "xor" if xor else "rlc", "fbn": fbn, "k": k, "r": r,
                          "src_hex": [s.tobytes().hex() for s in srcs], "ret": ret,
                          "rep_hex": [x.tobytes().hex() for x in rs], "repair_fpid_raw": fp})
    # precondition failures: r = 0 (RLC returns 1), XOR with r != 1
    pre = []
    for xor, k, r in [(False, 4, 0), (True, 4, 2), (True, 4, 0)]:
        srcs = [np.arange(10, dtype=np.uint8) + j for j in range(k)]
        ret, _, _ = R.encode_block(xor, 3, srcs, r)
        pre.append({"scheme": "xor" if xor else "rlc", "k": k, "r": r, "ret": ret})

    # ---- 3. Decode vectors --------------------------------------------------------------
    dec_cases = []

    def run_dec(xor, fbn, k, r, L, srcs_full, reps_full, src_mask, rep_mask, fpids, tag):
        srcs = [srcs_full[j] if src_mask[j] else None for j in range(k)]
        reps = [reps_full[i] if rep_mask[i] else None for i in range(r)]
        ret, rec = R.decode_block(xor, fbn, srcs, reps, fpids)
        d = {"tag": tag, "scheme": "xor" if xor else "rlc", "fbn": fbn, "k": k, "r": r, "L": L,
             "src_missing": [j for j in range(k) if not src_mask[j]],
             "rep_present": [i for i in range(r) if rep_mask[i]],
             "ret": ret, "crashed": ret <= -1000,
             "recovered": {str(j): sha(v.tobytes()) for j, v in sorted(rec.items())},
             "recovered_len": {str(j): int(len(v)) for j, v in sorted(rec.items())},
             "recovered_equals_original": all(
                 len(v) <= len(srcs_full[j]) + 4096 and
                 (v[: len(srcs_full[j])] == srcs_full[j]).all() and not v[len(srcs_full[j]):].any()
                 for j, v in rec.items())}
        return d

    drng = np.random.default_rng(99)
    for (k, r, L, e_list, ntrial, dseed) in [(4, 1, 1200, [1], 24, 31), (16, 4, 1200, [1, 2, 3, 4], 90, 32),
                                            (32, 8, 1200, [4, 8], 60, 33), (8, 8, 40, [1, 3, 5, 8], 120, 34),
                                            (64, 16, 9000, [16], 6, 35), (5, 3, 100, [1, 2, 3], 40, 36)]:
        for t in range(ntrial):
            fbn = int(drng.integers(0, 1 << 24))
            srcs_full = block_sources(dseed * 1000 + t, k, L)
            for xor in ([True, False] if r == 1 else [False]):
                ret, reps_full, fpids = R.encode_block(xor, fbn, srcs_full, r)
                assert ret == 0
                e = int(drng.choice(e_list))
                src_mask = np.ones(k, bool)
                src_mask[drng.choice(k, size=e, replace=False)] = False
                rep_mask = np.zeros(r, bool)
                mode = t % 3
                if mode == 0:       # exactly e repairs, the lowest-index ones
                    rep_mask[: min(e, r)] = True
                elif mode == 1:     # random subset of >= e repairs
                    n = int(drng.integers(min(e, r), r + 1))
                    rep_mask[drng.choice(r, size=n, replace=False)] = True
                else:               # random subset, possibly too few
                    n = int(drng.integers(0, r + 1))
                    rep_mask[drng.choice(r, size=n, replace=False)] = True
                dec_cases.append(run_dec(xor, fbn, k, r, L, srcs_full, reps_full, src_mask, rep_mask,
                                         fpids, f"k{k}r{r}L{L}_t{t}"))
                dec_cases[-1]["data_seed"] = dseed * 1000 + t

    # zero source symbols: the reference drops all-zero unknowns and everything that
    # depends on them (rlc_fec_scheme_gf256.c:98-101, 220-235)
    zero_cases = []
    zrng = np.random.default_rng(7)
    for t in range(40):
        k, r, L = 8, 4, 48
        srcs_full = [zrng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
        nz = int(zrng.integers(1, 3))
        for j in zrng.choice(k, size=nz, replace=False):
            srcs_full[j] = np.zeros(L, np.uint8)
        fbn = int(zrng.integers(0, 1 << 24))
        ret, reps_full, fpids = R.encode_block(False, fbn, srcs_full, r)
        e = int(zrng.integers(1, r + 1))
        src_mask = np.ones(k, bool)
        zeros = [j for j in range(k) if not srcs_full[j].any()]
        miss = set([int(zrng.choice(zeros))])
        while len(miss) < e:
            miss.add(int(zrng.integers(0, k)))
        for j in miss:
            src_mask[j] = False
        rep_mask = np.zeros(r, bool)
        rep_mask[zrng.choice(r, size=int(zrng.integers(e, r + 1)), replace=False)] = True
        d = run_dec(False, fbn, k, r, L, srcs_full, reps_full, src_mask, rep_mask, fpids, f"zero_t{t}")
        d["src_hex"] = [s.tobytes().hex() for s in srcs_full]
        zero_cases.append(d)

    # variable-length decode (sources shorter than the repair: zero padding; XOR too)
    vdec = []
    vrng = np.random.default_rng(55)
    for t in range(30):
        xor = t % 2 == 0
        k = int(vrng.integers(2, 9))
        r = 1 if xor else int(vrng.integers(1, 4))
        lens = [int(x) for x in vrng.integers(1, 1300, k)]
        srcs_full = [vrng.integers(0, 256, n, dtype=np.uint8) for n in lens]
        fbn = int(vrng.integers(0, 1 << 24))
        ret, reps_full, fpids = R.encode_block(xor, fbn, srcs_full, r)
        e = 1 if xor else int(vrng.integers(1, r + 1))
        src_mask = np.ones(k, bool)
        src_mask[vrng.choice(k, size=e, replace=False)] = False
        rep_mask = np.ones(r, bool)
        d = run_dec(xor, fbn, k, r, max(lens), srcs_full, reps_full, src_mask, rep_mask, fpids,
                    f"varlen_t{t}")
        d["src_hex"] = [s.tobytes().hex() for s in srcs_full]
        vdec.append(d)

    with open(os.path.join(OUT, "encode_cases.json"), "w") as f:
        json.dump({"generated_by": "tests/golden/gen_golden.py (reference pluglets, native gcc)",
                   "data": "oracle_py.synth_bytes(nblocks*k*L, data_seed) reshaped [block][k][L]",
                   "cases": enc_cases, "varlen": var_cases, "preconditions": pre}, f)
    np.savez_compressed(os.path.join(OUT, "encode_full.npz"), **arrays)
    with open(os.path.join(OUT, "decode_cases.json"), "w") as f:
        json.dump({"generated_by": "tests/golden/gen_golden.py (reference fec_recover in fork()ed child)",
                   "data": "sources = synth_bytes(k*L, data_seed) reshaped [k][L]; repairs = reference encode",
                   "cases": dec_cases, "zero_cases": zero_cases, "varlen_cases": vdec}, f)
    crashes = sum(c["crashed"] for c in dec_cases)
    print(f"encode cases {len(enc_cases)}, varlen {len(var_cases)}, decode {len(dec_cases)} "
          f"({crashes} reference crashes), zero {len(zero_cases)}, varlen-dec {len(vdec)}")
    window_cases(R)


def window_cases(R):
    """Sliding-window-shaped blocks (the framework every shipped FEC manifest composes:
    plugins/fec/fec.plugin:5-8, fec_rlc_gf256_window.plugin:5-8).

    Sender (window_framework_sender.h:209-250): the protected window is a block numbered 0
    (malloc_fec_block(cnx, 0), :215), so the reference encode seeds repair i with (0 << 8) | i;
    the repairs then leave with fec_block_number 0, symbol_number i and fec_scheme_specific = the
    window's first source id (:239-243).
    Receiver (window_framework_receiver.h:60-86): the block is numbered by that first source id
    (malloc_fec_block(cnx, source_symbol_id)) and repairs are slotted by symbol_number
    (fec.h:292-299); fec_recover seeds each equation with the repair's own FPID (:200) and stamps
    recovered sources (fec_block_number << 8) + j (:222).
    A few "mixed" blocks carry repairs whose FPID block numbers differ from each other (a peer
    is free to send them): the reference still seeds each equation by its own FPID."""
    out = []
    wrng = np.random.default_rng(4242)
    shapes = [(5, 1), (5, 2), (10, 3), (16, 4), (25, 5), (30, 5), (30, 10), (32, 8), (8, 8)]
    for t in range(160):
        k, r = shapes[t % len(shapes)]
        xor = r == 1 and t % 2 == 0
        varlen = t % 4 == 3
        L = 1200 if t % 3 else int(wrng.integers(1, 400)) * 4
        dseed = 70000 + t
        lens = [int(x) for x in wrng.integers(1, L + 1, k)] if varlen else None
        srcs_full = block_sources(dseed, k, L, lens)
        start = int(wrng.integers(0, 1 << 32)) if t % 5 else int(wrng.integers((1 << 32) - 64, 1 << 32))
        mixed = (not xor) and t % 11 == 7
        if mixed:  # every repair from a different block number: encode each one from its own block
            seed_fbn = [int(wrng.integers(0, 1 << 24)) for _ in range(r)]
            reps_full = []
            for i in range(r):
                ret, rs, _ = R.encode_block(False, seed_fbn[i], srcs_full, r)
                assert ret == 0
                reps_full.append(rs[i])
        else:
            seed_fbn = [0] * r
            ret, reps_full, _ = R.encode_block(xor, 0, srcs_full, r)   # window block number 0
            assert ret == 0
        fpids = [((seed_fbn[i] << 8) | i) | (start << 32) for i in range(r)]
        e = int(wrng.integers(1, min(r, k) + 1)) if not xor else 1
        src_mask = np.ones(k, bool)
        src_mask[wrng.choice(k, size=e, replace=False)] = False
        rep_mask = np.zeros(r, bool)
        if t % 3 == 0:
            rep_mask[: min(e, r)] = True
        else:
            rep_mask[wrng.choice(r, size=int(wrng.integers(min(e, r), r + 1)), replace=False)] = True
        srcs = [srcs_full[j] if src_mask[j] else None for j in range(k)]
        reps = [reps_full[i] if rep_mask[i] else None for i in range(r)]
        ret, rec, rfp = R.decode_block(xor, start, srcs, reps, fpids, with_fpids=True)
        d = {"tag": f"window_t{t}", "scheme": "xor" if xor else "rlc", "fbn": start, "k": k, "r": r, "L": L,
             "data_seed": dseed, "src_len": lens, "mixed_seeds": mixed, "repair_fpid_raw": fpids,
             "src_missing": [j for j in range(k) if not src_mask[j]],
             "rep_present": [i for i in range(r) if rep_mask[i]],
             "ret": ret, "crashed": ret <= -1000,
             "recovered": {str(j): sha(v.tobytes()) for j, v in sorted(rec.items())},
             "recovered_len": {str(j): int(len(v)) for j, v in sorted(rec.items())},
             "recovered_fpid": {str(j): int(f) for j, f in sorted(rfp.items())}}
        if not d["crashed"]:
            d["recovered_equals_original"] = all(
                (v[: len(srcs_full[j])] == srcs_full[j]).all() and not v[len(srcs_full[j]):].any()
                for j, v in rec.items())
        out.append(d)
    with open(os.path.join(OUT, "window_cases.json"), "w") as f:
        json.dump({"generated_by": "tests/golden/gen_golden.py window_cases (reference fec_recover in fork()ed "
                                   "child, window-framework-shaped blocks)",
                   "data": "sources = synth_bytes(k*L, data_seed) reshaped [k][L], truncated to src_len when given; "
                           "repairs = reference encode of block number 0 (per repair: of block number "
                           "repair_fpid_raw >> 8 & 0xffffff when mixed_seeds)",
                   "cases": out}, f)
    print(f"window cases {len(out)} ({sum(c['crashed'] for c in out)} reference crashes, "
          f"{sum(bool(c['recovered']) for c in out)} with recoveries)")


if __name__ == "__main__":
    main()
