#!/usr/bin/env python3
"""Generate pquic_amd/csrc/bitslice_gen.h -- the bitsliced GF(2^8) multiply-accumulate
engine of the RLC data path (gfx950 inline assembly).

How a lane computes  acc_i += c_ij * S_j  over GF(2^8)/0x11D for 32 bytes at a time
---------------------------------------------------------------------------------------
* Bit slicing.  The lane's 32 bytes of S_j (8 dwords w0..w7) are transposed with three
  rounds of masked shift-exchange (v_lshlrev/v_lshrrev + v_bitop3 mux) into 8 bit planes
  x_0..x_7: plane p holds bit p of all 32 bytes.  Multiplying every byte by a constant c
  is then a GF(2)-linear map on planes:  out_o = XOR_p M_c[o][p] x_p,  with column p of
  M_c = c * alpha^p.
* Four Russians.  Per source the lane builds TL[n] = XOR_{p<4, n_p} x_p and
  TH[n] = XOR_{p<4, n_p} x_{p+4} (n = 1..15, 22 XORs), so each output plane is ONE
  v_bitop3_b32 (3-input XOR):  acc_o ^= TL[row_o & 15] ^ TH[row_o >> 4].
  A coefficient therefore costs at most 8 full-rate VALU ops per 32 bytes.
* Dispatch.  The 8 register indices depend on the wave-uniform coefficient c, so the code
  is selected per coefficient from a shared table of 256 cases (80 bytes each, 64 KiB-aligned,
  entry 0 a return stub).  The case code names the accumulator planes as v0..v7;
  s_set_gpr_idx_on(SRC0,DST) relocates them to repair i's accumulators (ACC_BASE + 8 i), while
  the table operands (SRC1/SRC2) stay absolute.  Cases are CHAINED: the wrapper stages each
  source's coefficients as 16-bit case offsets ((c + 1) * 88, 0 = end), four to a 64-bit SGPR
  queue; the caller enters the first case with s_swappc_b64, and every case's tail advances M0
  by 8, shifts the queue, packs the next field under TAB's address bits and jumps straight to
  the next case (3 SALU + the branch) (the zero field lands on the stub,
  which returns).  One taken branch per coefficient instead of a call and a return; tiles with
  fewer live repairs (rt < RT) end their chain early.
* Output.  The same three exchange rounds are an involution, so applying them to the
  accumulator planes yields the repair bytes in the original word order.

The generator self-checks the plane algebra and the transpose against a byte-level GF
model before writing the header.
"""
from __future__ import annotations

import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.environ.get("FEC_GEN_OUT") or os.path.join(HERE, "bitslice_gen.h")

# ----------------------------------------------------------------------------- register map
# T64: the exchange rounds shift two words per instruction (v_lshlrev_b64 / v_lshrrev_b64 on an
# aligned register pair) -- 36 VALU per transpose instead of 48.  The pairs a 64-bit shift takes
# must be adjacent, so a lane's 8 words and a repair's 8 accumulator planes sit in the slot order
# SIG (self-inverse: slot s holds logical word / plane SIG[s]), round 0 writes an 8-register
# scratch block in natural order, round 1 runs in place there, round 2 writes the destination.
T64 = os.environ.get("FEC_GEN_T64", "1") != "0"
SIG64 = [0, 2, 1, 3, 4, 6, 5, 7]
SIG = SIG64 if T64 else list(range(8))
TAIL_HH = os.environ.get("FEC_GEN_TAIL_HH", "0") != "0"
# AB: two case tables in one 64 KiB window.  Table A (offset 0) holds the cases of even chain
# positions, table B (offset TABLE_B) those of odd positions, with the accumulators 8 registers
# further on.  An A case takes its successor from queue QB (s[S_C2:S_C3]), a B case from queue QA
# (s[S_C0:S_C1]) and advances M0 by 16: two SALU per A case, three per B case (three each without
# AB), and the two 64-bit queues hold 8 fields, so an 8-repair tile is one chain (two without AB).
AB = os.environ.get("FEC_GEN_AB", "0") != "0"
TABLE_B = 32768
# EARLY_PF: the register-prefetch bodies refill a source buffer right after round 0 of its transpose
# (P sources in flight, the load issued ~1 step earlier) instead of at the start of the next step
EARLY_PF = T64 and os.environ.get("FEC_GEN_EARLY_PF", "1") != "0"
# EARLY_CO (with EARLY_PF): a step's coefficient fields are read before its transpose, not after
EARLY_CO = os.environ.get("FEC_GEN_EARLY_CO", "0") != "0"
# register-prefetch bodies compute exec-masked to the lanes that own pieces (vm0: at L = 1200, 38 of
# 64), as the ring bodies do; idle lanes then neither load nor switch
EXECMASK = os.environ.get("FEC_GEN_EXECMASK", "0") != "0"
# TOUCH (decode register bodies, EARLY_PF): after each row's loads, one dword load per lane 32 bytes
# apart over the row TOUCH - 1 rows beyond it (an L2 warm-up of a row not yet in flight; the data is
# dropped).  Costs 4 VGPRs above the accumulators and one VMEM per row in the vmcnt budget
TOUCH = int(os.environ.get("FEC_GEN_TOUCH", "0"))
# DEC_EPI_PF (decode register bodies): the epilogue reads each output address one row ahead, so no
# LDS round trip is waited for per recovered row (before: one per row plus one for the row count)
DEC_EPI_PF = os.environ.get("FEC_GEN_DEC_EPI_PF", "0") != "0"


def table_map(B):
    """Four-Russians table registers from B: the planes (singletons 1, 2, 4, 8 of TL and TH) at
    B..B+7, the 22 combinations at B+8..B+29."""
    tl = {1: B, 2: B + 1, 4: B + 2, 8: B + 3}
    th = {1: B + 4, 2: B + 5, 4: B + 6, 8: B + 7}
    for i, n in enumerate([3, 5, 6, 7, 9, 10, 11, 12, 13, 14, 15]):
        tl[n] = B + 8 + i
        th[n] = B + 19 + i
    return tl, th


T_BASE = 32
if T64:
    TL, TH = table_map(T_BASE)                           # v32..v61
else:
    TL = {n: T_BASE + n - 1 for n in range(1, 16)}      # v32..v46
    TH = {n: T_BASE + 15 + n - 1 for n in range(1, 16)}  # v47..v61
TMP = [62, 63, 64, 65]
CO = TMP  # coefficient fields: read into the transpose temporaries once the transpose is done
COPTR = 66
INPTR = 67   # decode only: next entry of the input-address table
OUTPTR = 68  # decode only
NADDR = 70   # decode only: the next source's address, read from the table one source ahead
DATA_BASE = 68  # encode; decode data buffers start at 70 (tuples must start on an even VGPR)
CASE_BYTES = 80  # <= 8 VOP3 (64 B) + the 16-byte chain tail; table entry 0 is the return stub
V1_TABLE = "fec_bs_case_table"
# stage-0 destinations (scratch, overwritten by the combos), stage-2 destinations (planes)
XS = [TL[3], TL[5], TL[6], TL[7], TH[3], TH[5], TH[6], TH[7]]
PL = [TL[1], TL[2], TL[4], TL[8], TH[1], TH[2], TH[4], TH[8]]
# SGPRs owned by the asm bodies
S_TAB, S_TGT, S_RET, S_TABHI, S_J = 60, 62, 64, 66, 67  # S_TABHI = TAB.lo >> 16
S_C = [68, 69, 70, 71]  # coefficient-field dwords of the current source (readfirstlane of CO)
S_CQ = 84        # chain queue: the remaining 16-bit case offsets of the running chain (shared with
                 # the decode epilogue's exec save, which never overlaps a chain)
S_MASK = [72, 73, 74]
S_T2 = 75
S_CUR = 76
S_SAVEM0 = 78
S_RT = 79
S_SAVEEX = 80
S_OUT = 82
S_T3 = 84
S_EPI = 86
S_S = 88
S_JL = 89        # enc: sources loaded in the current block (the prefetch crosses block boundaries)
S_O2 = 90
S_DJ = 92        # enc: pointer jump applied when a block's last source has been loaded
SGPR_CLOBBER = list(range(60, 94))  # s0-s59 and s94-s101 stay with the compiler
MASKS = [0x55555555, 0x33333333, 0x0F0F0F0F]
STAGES = [  # (shift, mask index, pairs)
    (1, 0, [(0, 1), (2, 3), (4, 5), (6, 7)]),
    (2, 1, [(0, 2), (1, 3), (4, 6), (5, 7)]),
    (4, 2, [(0, 4), (1, 5), (2, 6), (3, 7)]),
]


# ----------------------------------------------------------------------------- GF model
def gf_mul(a: int, b: int) -> int:
    p = 0
    for _ in range(8):
        if b & 1:
            p ^= a
        b >>= 1
        carry = a & 0x80
        a = (a << 1) & 0xFF
        if carry:
            a ^= 0x1D
    return p


def case_rows(c: int):
    """(nl, nh) per output plane o for coefficient c."""
    col = [gf_mul(c, 1 << p) for p in range(8)]  # column p = c * alpha^p
    rows = []
    for o in range(8):
        bits = [(col[p] >> o) & 1 for p in range(8)]
        nl = sum(bits[p] << p for p in range(4))
        nh = sum(bits[p + 4] << p for p in range(4))
        rows.append((nl, nh))
    return rows


def selfcheck():
    # plane algebra: out byte = c * x for every c, x
    for c in range(256):
        rows = case_rows(c)
        for x in range(256):
            xp = [(x >> p) & 1 for p in range(8)]
            tl = lambda n: sum(xp[p] for p in range(4) if (n >> p) & 1) & 1  # noqa: E731
            th = lambda n: sum(xp[p + 4] for p in range(4) if (n >> p) & 1) & 1  # noqa: E731
            out = 0
            for o, (nl, nh) in enumerate(rows):
                out |= (tl(nl) ^ th(nh)) << o
            assert out == gf_mul(c, x), (c, x)
    # transpose: plane p = bit p of all 32 bytes; involution
    rnd = random.Random(1)
    for _ in range(200):
        w = [rnd.getrandbits(32) for _ in range(8)]
        t = transpose_model(w)
        for p in range(8):
            for byte in range(4):
                for b in range(8):
                    orig = (w[b] >> (8 * byte + p)) & 1
                    assert ((t[p] >> (8 * byte + b)) & 1) == orig
        assert transpose_model(t) == w


def transpose_model(w):
    w = list(w)
    for sh, mi, pairs in STAGES:
        m = MASKS[mi]
        for a, b in pairs:
            t0 = (w[b] << sh) & 0xFFFFFFFF
            t1 = w[a] >> sh
            na = (m & w[a]) | (~m & t0 & 0xFFFFFFFF)
            nb = (m & t1) | (~m & w[b] & 0xFFFFFFFF)
            w[a], w[b] = na, nb
    return w


# ----------------------------------------------------------------------------- code emitters
def v(n):
    return f"v{n}"


def inline_cases(RT, tl, th, acc_base, c):
    """FEC_GEN_INLINE_CASES=c (timing probes only, results are garbage): RT case bodies of the fixed
    coefficient c inline, no jump.  FEC_GEN_INLINE_MODE: 'plain' (absolute accumulators), 'salu' (plus the
    three SALU of a chain tail per case, on dead SGPRs), 'idx' (GPR-index mode on, M0 advanced per case,
    as the chains run): what the dispatch's jumps, tail SALU and index mode each cost."""
    mode = os.environ.get("FEC_GEN_INLINE_MODE", "plain")
    out = []
    if mode == "idx":
        out.append(f"s_set_gpr_idx_on {acc_base}, gpr_idx(SRC0,DST)")
    for i in range(RT):
        for o, (nl, nh) in enumerate(case_rows(c)):
            s = SIG[o] if mode == "idx" else acc_base + 8 * i + SIG[o]
            if nl and nh:
                out.append(f"v_bitop3_b32 v{s}, v{s}, {v(tl[nl])}, {v(th[nh])} bitop3:0x96")
            elif nl:
                out.append(f"v_xor_b32 v{s}, v{s}, {v(tl[nl])}")
            elif nh:
                out.append(f"v_xor_b32 v{s}, v{s}, {v(th[nh])}")
        if mode == "idx":
            out.append("s_add_u32 m0, m0, 8")
        elif mode == "salu":
            out += [f"s_add_u32 s{S_TGT + 1}, s{S_TGT + 1}, 8",
                    f"s_lshr_b64 s[{S_CQ}:{S_CQ + 1}], s[{S_CQ}:{S_CQ + 1}], 16",
                    f"s_pack_ll_b32_b16 s{S_TGT}, s{S_CQ}, s{S_TABHI}"]
    if mode == "idx":
        out.append("s_set_gpr_idx_off")
    return out


def emit_table(sym="fec_bs_case_table", tl=None, th=None):
    tl = tl or TL
    th = th or TH
    lines = ['  .text', '  .p2align 16', f'  .globl {sym}', f'  .hidden {sym}', f'{sym}:']
    # entry 0: the chain's end (a zero field) returns to the caller
    lines.append(f"  s_setpc_b64 s[{S_RET}:{S_RET + 1}]")
    lines.append(f"  .org {sym} + {CASE_BYTES}")
    if AB:
        assert not TAIL_HH and TABLE_B + 257 * CASE_BYTES <= 65536
        for half, base in ((0, 0), (1, TABLE_B)):
            if half:
                lines.append(f"  .org {sym} + {TABLE_B}")
                lines.append(f"  s_setpc_b64 s[{S_RET}:{S_RET + 1}]")
            for c in range(256):
                lines.append(f"  .org {sym} + {base + CASE_BYTES * (c + 1)}")
                body = []
                for o, (nl, nh) in enumerate(case_rows(c)):
                    d = 8 * half + SIG[o]
                    if nl and nh:
                        body.append(f"v_bitop3_b32 v{d}, v{d}, {v(tl[nl])}, {v(th[nh])} bitop3:0x96")
                    elif nl:
                        body.append(f"v_xor_b32 v{d}, v{d}, {v(tl[nl])}")
                    elif nh:
                        body.append(f"v_xor_b32 v{d}, v{d}, {v(th[nh])}")
                q = S_C[0] if half else S_C[2]  # successor: an A case's is in QB, a B case's in QA
                body += [f"s_pack_ll_b32_b16 s{S_TGT}, s{q}, s{S_TABHI}",
                         f"s_lshr_b64 s[{q}:{q + 1}], s[{q}:{q + 1}], 16"]
                if half:
                    body.append("s_add_u32 m0, m0, 16")
                body.append(f"s_setpc_b64 s[{S_TGT}:{S_TGT + 1}]")
                lines += ["  " + b for b in body]
        lines.append(f"  .org {sym} + {TABLE_B + CASE_BYTES * 257}")
        return lines
    for c in range(256):
        body = []
        for o, (nl, nh) in enumerate(case_rows(c)):
            s = SIG[o]  # plane o's accumulator slot
            if nl and nh:
                body.append(f"v_bitop3_b32 v{s}, v{s}, {v(tl[nl])}, {v(th[nh])} bitop3:0x96")
            elif nl:
                body.append(f"v_xor_b32 v{s}, v{s}, {v(tl[nl])}")
            elif nh:
                body.append(f"v_xor_b32 v{s}, v{s}, {v(th[nh])}")
        # chain tail: next repair's accumulators, next 16-bit case offset, jump (entry 0 returns)
        if TAIL_HH:  # the next offset is the queue's second field: packed before the shift, so the
            # jump waits on one SALU result instead of two (TAB.lo[31:16] comes from S_TAB itself)
            body += [f"s_pack_hh_b32_b16 s{S_TGT}, s{S_CQ}, s{S_TAB}",
                     f"s_lshr_b64 s[{S_CQ}:{S_CQ + 1}], s[{S_CQ}:{S_CQ + 1}], 16",
                     f"s_add_u32 m0, m0, 8",
                     f"s_setpc_b64 s[{S_TGT}:{S_TGT + 1}]"]
        else:
            body += [f"s_add_u32 m0, m0, 8",
                     f"s_lshr_b64 s[{S_CQ}:{S_CQ + 1}], s[{S_CQ}:{S_CQ + 1}], 16",
                     f"s_pack_ll_b32_b16 s{S_TGT}, s{S_CQ}, s{S_TABHI}",
                     f"s_setpc_b64 s[{S_TGT}:{S_TGT + 1}]"]
        lines += ["  " + b for b in body]
        lines.append(f"  .org {sym} + {CASE_BYTES * (c + 2)}")
    return lines


def transpose_fwd(src_words):
    """src_words: 8 VGPR numbers (read only). Writes planes into PL via scratch XS."""
    out = []
    cur = list(src_words)
    for si, (sh, mi, pairs) in enumerate(STAGES):
        dst = list(cur)
        for pi, (a, b) in enumerate(pairs):
            if si == 0:
                da, db = XS[a], XS[b]
            elif si == 2:
                da, db = PL[a], PL[b]
            else:
                da, db = cur[a], cur[b]
            t0, t1 = (TMP[0], TMP[1]) if pi % 2 == 0 else (TMP[2], TMP[3])
            out += [f"v_lshlrev_b32 v{t0}, {sh}, v{cur[b]}",
                    f"v_lshrrev_b32 v{t1}, {sh}, v{cur[a]}",
                    f"v_bitop3_b32 v{da}, s{S_MASK[mi]}, v{cur[a]}, v{t0} bitop3:0xca",
                    f"v_bitop3_b32 v{db}, s{S_MASK[mi]}, v{t1}, v{cur[b]} bitop3:0xca"]
            dst[a], dst[b] = da, db
        cur = dst
    return out


def transpose_inplace(regs, tmp=None):
    """The three exchange rounds on 8 registers in place (an involution: words <-> bit planes).
    tmp: 4 temporaries (two pairs, so consecutive exchanges overlap) or 2 (one pair)."""
    tmp = tmp or TMP
    out = []
    for sh, mi, pairs in STAGES:
        for pi, (a, b) in enumerate(pairs):
            t0, t1 = (tmp[0], tmp[1]) if pi % 2 == 0 or len(tmp) < 4 else (tmp[2], tmp[3])
            out += [f"v_lshlrev_b32 v{t0}, {sh}, v{regs[b]}",
                    f"v_lshrrev_b32 v{t1}, {sh}, v{regs[a]}",
                    f"v_bitop3_b32 v{regs[a]}, s{S_MASK[mi]}, v{regs[a]}, v{t0} bitop3:0xca",
                    f"v_bitop3_b32 v{regs[b]}, s{S_MASK[mi]}, v{t1}, v{regs[b]} bitop3:0xca"]
    return out


def t64_scratch(B):
    """T64 scratch of a table map based at B: 8 consecutive registers for rounds 0-1 and two
    register pairs of shift temporaries, all among the combination registers (dead between a
    block's last case and the next source's combos; clear of the ring decode epilogue's B+8..B+12)."""
    return list(range(B + 14, B + 22)), list(range(B + 22, B + 26))


def transpose64(inp, out, X, T):
    """The three exchange rounds with 64-bit shifts (36 VALU).  inp[w]: register of logical word
    (or plane) w, with (inp[0], inp[2]), (inp[1], inp[3]), (inp[4], inp[6]), (inp[5], inp[7]) aligned
    register pairs; out[p]: destination of plane (or word) p (may alias inp); X: 8 consecutive
    scratch registers (aligned); T: 4 temporaries (two aligned pairs).
    A 64-bit shift moves the low word's top bits into the high word's low bits (left) or the high
    word's low bits into the low word's top bits (right); every mask keeps the other operand
    there (its low s bits are set, its top s bits clear), so those bits never reach a result."""
    assert X[0] % 2 == 0 and X == list(range(X[0], X[0] + 8))
    assert T[0] % 2 == 0 and T[1] == T[0] + 1 and T[2] % 2 == 0 and T[3] == T[2] + 1
    for h in (0, 4):
        for a, b in ((h, h + 2), (h + 1, h + 3)):
            assert inp[a] % 2 == 0 and inp[b] == inp[a] + 1, (inp, a, b)
    assert not set(X) & set(inp) and not set(T) & (set(inp) | set(X))
    m = [f"s{S_MASK[i]}" for i in range(3)]
    mux = lambda d, sel, x, y: f"v_bitop3_b32 v{d}, {sel}, v{x}, v{y} bitop3:0xca"  # noqa: E731
    tb, ta = T[0], T[2]
    L = []
    for h in (0, 4):  # round 0 (shift 1): pairs (h, h+1), (h+2, h+3); inp -> X
        L += [f"v_lshlrev_b64 v[{tb}:{tb + 1}], 1, v[{inp[h + 1]}:{inp[h + 1] + 1}]",
              f"v_lshrrev_b64 v[{ta}:{ta + 1}], 1, v[{inp[h]}:{inp[h] + 1}]",
              mux(X[h], m[0], inp[h], tb), mux(X[h + 1], m[0], ta, inp[h + 1]),
              mux(X[h + 2], m[0], inp[h + 2], tb + 1), mux(X[h + 3], m[0], ta + 1, inp[h + 3])]
    for h in (0, 4):  # round 1 (shift 2): pairs (h, h+2), (h+1, h+3); in place in X
        L += [f"v_lshlrev_b64 v[{tb}:{tb + 1}], 2, v[{X[h + 2]}:{X[h + 3]}]",
              f"v_lshrrev_b64 v[{ta}:{ta + 1}], 2, v[{X[h]}:{X[h + 1]}]",
              mux(X[h], m[1], X[h], tb), mux(X[h + 1], m[1], X[h + 1], tb + 1),
              mux(X[h + 2], m[1], ta, X[h + 2]), mux(X[h + 3], m[1], ta + 1, X[h + 3])]
    for g in (0, 2):  # round 2 (shift 4): pairs (g, g+4), (g+1, g+5); X -> out
        L += [f"v_lshlrev_b64 v[{tb}:{tb + 1}], 4, v[{X[g + 4]}:{X[g + 5]}]",
              f"v_lshrrev_b64 v[{ta}:{ta + 1}], 4, v[{X[g]}:{X[g + 1]}]",
              mux(out[g], m[2], X[g], tb), mux(out[g + 1], m[2], X[g + 1], tb + 1),
              mux(out[g + 4], m[2], ta, X[g + 4]), mux(out[g + 5], m[2], ta + 1, X[g + 5])]
    return L


def simulate(lines, regs):
    """Run the exchange-round instructions of `lines` on a {vgpr: u32} register file (self-check)."""
    import re
    M = 0xFFFFFFFF
    smask = {f"s{S_MASK[i]}": MASKS[i] for i in range(3)}
    for ln in lines:
        p = re.match(r"v_(lshl|lshr)rev_b64 v\[(\d+):(\d+)\], (\d+), v\[(\d+):(\d+)\]", ln)
        if p:
            d, s, x = int(p.group(2)), int(p.group(4)), int(p.group(5))
            val = regs[x] | (regs[x + 1] << 32)
            val = (val << s) if p.group(1) == "lshl" else (val >> s)
            regs[d], regs[d + 1] = val & M, (val >> 32) & M
            continue
        p = re.match(r"v_(lshl|lshr)rev_b32 v(\d+), (\d+), v(\d+)", ln)
        if p:
            s, x = int(p.group(3)), regs[int(p.group(4))]
            regs[int(p.group(2))] = ((x << s) if p.group(1) == "lshl" else (x >> s)) & M
            continue
        p = re.match(r"v_bitop3_b32 v(\d+), (s\d+), v(\d+), v(\d+) bitop3:0xca", ln)
        assert p, ln
        mk, a, b = smask[p.group(2)], regs[int(p.group(3))], regs[int(p.group(4))]
        regs[int(p.group(1))] = ((mk & a) | (~mk & b)) & M
    return regs


def selfcheck_t64():
    """transpose64 as the bodies call it: words loaded in slot order SIG -> planes; planes in
    accumulator slots SIG -> words back in their load slots; and the transpose_inplace twin."""
    rnd = random.Random(2)
    base, X, T = 100, list(range(120, 128)), list(range(130, 134))
    fwd = transpose64([base + SIG64[w] for w in range(8)], list(range(140, 148)), X, T)
    inv = transpose64([base + SIG64[o] for o in range(8)], [base + SIG64[w] for w in range(8)], X, T)
    for _ in range(200):
        phys = [rnd.getrandbits(32) for _ in range(8)]  # slot s holds logical word SIG64[s]
        words = [phys[SIG64[w]] for w in range(8)]
        regs = {r: rnd.getrandbits(32) for r in range(100, 150)}
        regs.update({base + s: phys[s] for s in range(8)})
        simulate(fwd, regs)
        assert [regs[140 + p] for p in range(8)] == transpose_model(words)
        regs.update({base + SIG64[o]: transpose_model(words)[o] for o in range(8)})
        simulate(inv, regs)
        assert [regs[base + s] for s in range(8)] == phys


def combos(tl=None, th=None):
    out = []
    for T in (tl or TL, th or TH):
        out += [f"v_xor_b32 v{T[3]}, v{T[1]}, v{T[2]}",
                f"v_xor_b32 v{T[5]}, v{T[1]}, v{T[4]}",
                f"v_xor_b32 v{T[6]}, v{T[2]}, v{T[4]}",
                f"v_xor_b32 v{T[9]}, v{T[1]}, v{T[8]}",
                f"v_xor_b32 v{T[10]}, v{T[2]}, v{T[8]}",
                f"v_xor_b32 v{T[12]}, v{T[4]}, v{T[8]}",
                f"v_bitop3_b32 v{T[7]}, v{T[1]}, v{T[2]}, v{T[4]} bitop3:0x96",
                f"v_bitop3_b32 v{T[11]}, v{T[1]}, v{T[2]}, v{T[8]} bitop3:0x96",
                f"v_bitop3_b32 v{T[13]}, v{T[1]}, v{T[4]}, v{T[8]} bitop3:0x96",
                f"v_bitop3_b32 v{T[14]}, v{T[2]}, v{T[4]}, v{T[8]} bitop3:0x96",
                f"v_bitop3_b32 v{T[15]}, v{T[3]}, v{T[4]}, v{T[8]} bitop3:0x96"]
    return out


LOADOP = {16: ("global_load_dwordx4", "global_store_dwordx4", 4),
          8: ("global_load_dwordx2", "global_store_dwordx2", 2),
          4: ("global_load_dword", "global_store_dword", 1)}


def coef_row_bytes(RT: int) -> int:
    """LDS bytes per source of a coefficient row: max(4, RT) little-endian u16 fields, field i =
    (c_i + 1) * CASE_BYTES (the case's offset in the table), 0 = end of chain."""
    return 2 * max(4, RT)


def regrange(base, n):
    return f"v{base}" if n == 1 else f"v[{base}:{base + n - 1}]"


def body(mode: str, RT: int, VEC: int, P: int, sc: bool = False):
    """Inline-asm text for one group of blocks x one column chunk.

    The sources of all blocks of the group form ONE stream (flattened index s = g*k + j),
    so the P-deep register prefetch runs across block boundaries; when j wraps, the
    per-block epilogue subroutine (reached by s_swappc) transposes the accumulators back,
    stores them and clears them.  mode 'enc' (addresses by stride) or 'dec' (addresses
    from LDS tables written by the wrapper)."""
    ld, st, nw = LOADOP[VEC]
    NP = 32 // VEC
    DATA_BASE = data_base(mode)
    acc_base = DATA_BASE + 8 * P
    touch = TOUCH if mode == "dec" and EARLY_PF else 0
    epi_pf = mode == "dec" and DEC_EPI_PF and T64
    EPI_RT, EPI_AD = PL[0], PL[2]  # v32, v34:35 (planes, dead in the epilogue; clear of t64 scratch)
    assert not epi_pf or (EPI_AD % 2 == 0 and EPI_AD + 1 == PL[3] and {EPI_RT, EPI_AD, EPI_AD + 1}.isdisjoint(
        set(sum(t64_scratch(T_BASE), []))))
    TA = acc_base + 8 * RT  # touch: the row address (pair), the dropped data, the lane offset
    TD, TOFF = TA + 2, TA + 3
    assert acc_base + 8 * RT + (4 if touch else 0) <= 256
    assert not touch or (touch >= 2 and (NP + 1) * (P - 1) + 1 <= 63)
    L = []
    a = L.append
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    a(f"s_mov_b32 s{S_SAVEM0}, m0")
    a(f"s_mov_b64 s[{S_SAVEEX}:{S_SAVEEX + 1}], exec")
    live = "%[vm0]" if EXECMASK else f"s[{S_SAVEEX}:{S_SAVEEX + 1}]"  # exec of the compute
    if EXECMASK:
        a(f"s_mov_b64 exec, {live}")
    for i, m in enumerate(MASKS):
        a(f"s_mov_b32 s{S_MASK[i]}, 0x{m:08x}")
    a(f"s_getpc_b64 s[{S_TAB}:{S_TAB + 1}]")
    a(f"s_add_u32 s{S_TAB}, s{S_TAB}, {V1_TABLE}@rel32@lo+4")
    a(f"s_addc_u32 s{S_TAB + 1}, s{S_TAB + 1}, {V1_TABLE}@rel32@hi+12")
    # the table is 64 KiB-aligned and 20 KiB long: a target is TAB's upper 48 bits with the case
    # offset as its low 16 (s_pack_ll of the queue field and TAB.lo >> 16); the engine checks the
    # alignment on the device before the first launch (fec_bs_case_table_addr)
    a(f"s_lshr_b32 s{S_TABHI}, s{S_TAB}, 16")
    a(f"s_mov_b32 s{S_TGT + 1}, s{S_TAB + 1}")
    a(f"s_getpc_b64 s[{S_EPI}:{S_EPI + 1}]")
    a(".Lepipc_%=:")
    a(f"s_add_u32 s{S_EPI}, s{S_EPI}, .Lepi_%= - .Lepipc_%=")
    a(f"s_addc_u32 s{S_EPI + 1}, s{S_EPI + 1}, 0")
    for r in range(acc_base, acc_base + 8 * RT):
        a(f"v_mov_b32 v{r}, 0")
    for r in range(DATA_BASE, DATA_BASE + 8 * P):
        a(f"v_mov_b32 v{r}, 0")
    a(f"v_mov_b32 v{COPTR}, %[coef]")
    if AB and coef_row_bytes(RT) == 8:  # rows of 4 fields: QA / QB are one dword each
        a(f"s_mov_b32 s{S_C[1]}, 0")
        a(f"s_mov_b32 s{S_C[3]}, 0")
    if mode == "enc":
        a(f"s_mov_b64 s[{S_CUR}:{S_CUR + 1}], %[src]")
        a(f"s_mov_b64 s[{S_OUT}:{S_OUT + 1}], %[rep]")
    else:
        a(f"v_mov_b32 v{INPTR}, %[intab]")
        a(f"ds_read_b64 v[{NADDR}:{NADDR + 1}], v{INPTR}")  # source 0's address
        if touch:  # row touch - 1's address, touched after source 0's loads
            a(f"ds_read_b64 v[{TA}:{TA + 1}], v{INPTR} offset:{8 * (touch - 1)}")
            a(f"v_lshlrev_b32 v{TOFF}, {NP.bit_length() - 1}, %[off0]")  # lane * 32 (0 on idle lanes)
            # S_JL = rows with a touch target (y + touch - 1 < nsrc for the y-th row loaded)
            a(f"s_sub_u32 s{S_JL}, %[nsrc], {touch - 1}")
            a(f"s_cselect_b32 s{S_JL}, 0, s{S_JL}")
        a(f"v_add_u32 v{INPTR}, 8, v{INPTR}")
        a(f"v_mov_b32 v{OUTPTR}, %[outtab]")
    # count-down loop counters, tested by the borrow of s_sub_u32 (no compares in the loop):
    # S_S = sources left after this one, S_J = sources left in this block after this one,
    # S_T2 = prefetches left (max(0, nsrc - (P - 1)))
    a(f"s_sub_u32 s{S_S}, %[nsrc], 1")
    a(f"s_sub_u32 s{S_J}, %[k], 1")
    a(f"s_sub_u32 s{S_T2}, %[nsrc], {P if EARLY_PF else P - 1}")
    a(f"s_cselect_b32 s{S_T2}, 0, s{S_T2}")
    if mode == "enc":
        a(f"s_mov_b32 s{S_JL}, 0")

    def load_source(buf, lgkm=0):
        out = []
        if mode == "dec":
            # this source's address was read one source ago (nothing else of the LDS queue is
            # outstanding here but, with EARLY_CO, this step's younger coefficient read, so the
            # wait is free); then fetch the next one
            out += [f"s_waitcnt lgkmcnt({lgkm})",
                    f"v_readfirstlane_b32 s{S_CUR}, v{NADDR}",
                    f"v_readfirstlane_b32 s{S_CUR + 1}, v{NADDR + 1}",
                    f"ds_read_b64 v[{NADDR}:{NADDR + 1}], v{INPTR}"]
            if touch:  # the touch target read one row ago, and the next one's address
                out += [f"v_readfirstlane_b32 s{S_O2}, v{TA}",
                        f"v_readfirstlane_b32 s{S_O2 + 1}, v{TA + 1}",
                        f"ds_read_b64 v[{TA}:{TA + 1}], v{INPTR} offset:{8 * (touch - 1)}"]
            out += [f"v_add_u32 v{INPTR}, 8, v{INPTR}"]
        # no exec switching: a lane's piece past the chunk end has offset 0 (BsLanes), so its load
        # stays inside the row, and its bytes never reach memory (the stores are masked)
        for q in range(NP):
            out.append(f"{ld} {regrange(DATA_BASE + 8 * buf + q * nw, nw)}, %[off{q}], s[{S_CUR}:{S_CUR + 1}]@LDPOL@")
        if touch:
            # past the last target the touch re-reads this row (every row's loads are followed by
            # exactly one touch, which the vmcnt waits count); the selects leave S_O2 SALU-written
            out += [f"s_sub_u32 s{S_JL}, s{S_JL}, 1",
                    f"s_cselect_b64 s[{S_O2}:{S_O2 + 1}], s[{S_CUR}:{S_CUR + 1}], s[{S_O2}:{S_O2 + 1}]",
                    f"s_cselect_b32 s{S_JL}, 0, s{S_JL}",
                    f"global_load_dword v{TD}, v{TOFF}, s[{S_O2}:{S_O2 + 1}]"]
        if mode == "enc":
            # next row of this block, or -- after its k-th row -- the first row of the group's next
            # block, which starts bstep blocks further on: one 64-bit select between the two steps
            # (%[ll] = L, %[sdl] = L + delta), through the chain queue (idle while loads issue)
            out += [f"s_add_u32 s{S_JL}, s{S_JL}, 1",
                    f"s_cmp_eq_u32 s{S_JL}, %[k]",
                    f"s_cselect_b64 s[{S_CQ}:{S_CQ + 1}], %[sdl], %[ll]",
                    f"s_cselect_b32 s{S_JL}, 0, s{S_JL}",
                    f"s_add_u32 s{S_CUR}, s{S_CUR}, s{S_CQ}",
                    f"s_addc_u32 s{S_CUR + 1}, s{S_CUR + 1}, s{S_CQ + 1}"]
        return out

    for q in range(P if EARLY_PF else P - 1):  # prologue: sources 0 .. P-1 (P-2 without EARLY_PF)
        a(f"s_cmp_lt_u32 {q}, %[nsrc]")
        a(f"s_cbranch_scc0 .Lpro_done_%=")
        L.extend(load_source(q))
    a(".Lpro_done_%=:")
    csb = coef_row_bytes(RT)  # per source: max(4, RT) 16-bit case offsets
    dsr = "ds_read_b64" if csb == 8 else "ds_read_b128"
    ndw = min(4, csb // 4)
    nch = max(1, RT // 4)  # chains of up to 4 cases (one 64-bit queue each)
    # the common path of every source step falls through: the prefetch-less tail steps and the
    # block-end epilogue calls are out of line (after the loop), so a step costs no taken branch
    # besides its case chains
    ool = []
    early_co = EARLY_PF and EARLY_CO and csb <= 16 and not os.environ.get("FEC_GEN_CONSTCOEF")
    for b in range(P):
        nb = (b + P - 1) % P
        a(f".Lbody{b}_%=:")
        a(f"s_sub_u32 s{S_T2}, s{S_T2}, 1")
        a(f"s_cbranch_scc1 .Lnopf{b}_%=")
        if EARLY_PF:
            # source s waits in buffer b; P sources are in flight.  Round 0 of the transpose is the
            # buffer's only reader, so source s + P is loaded into it right after (SCC still holds
            # the borrow of the S_T2 decrement: VALU and s_waitcnt leave it alone)
            # with touches: each younger row brings NP + 1 loads, and this row's own touch follows it
            a(f"s_waitcnt vmcnt({(NP + 1) * (P - 1) + 1 if touch else NP * (P - 1)})")
            a(f".Lpf{b}_%=:")
            ool += [f".Lnopf{b}_%=:", f"s_mov_b32 s{S_T2}, 0", "s_waitcnt vmcnt(0)", f"s_branch .Lpf{b}_%="]
            tr = transpose64([DATA_BASE + 8 * b + SIG[w] for w in range(8)], PL, *t64_scratch(T_BASE))
            if os.environ.get("FEC_GEN_PROBE_NOTRANS"):  # timing probe only (garbage): no forward transpose
                tr = []
            if early_co:  # the coefficient fields (into CO = TMP, untouched by transpose64) go out first
                a(f"{dsr} {regrange(CO[0], ndw)}, v{COPTR}")
                a(f"v_add_u32 v{COPTR}, {csb}, v{COPTR}")
            L.extend(tr[:12])
            a(f"s_cbranch_scc1 .Lnold{b}_%=")
            L.extend(load_source(b, 1 if early_co else 0))
            a(f".Lnold{b}_%=:")
            L.extend(tr[12:])
        else:
            L.extend(load_source(nb))
            # FEC_GEN_NOVMWAIT=1 (timing probe only, results are garbage): no wait for the source rows
            a(f"s_waitcnt vmcnt({63 if os.environ.get('FEC_GEN_NOVMWAIT') else NP * (P - 1)})")
            a(f".Lpf{b}_%=:")
            ool += [f".Lnopf{b}_%=:", f"s_mov_b32 s{S_T2}, 0", "s_waitcnt vmcnt(0)", f"s_branch .Lpf{b}_%="]
            if T64:
                L.extend(transpose64([DATA_BASE + 8 * b + SIG[w] for w in range(8)], PL, *t64_scratch(T_BASE)))
            else:
                L.extend(transpose_fwd([DATA_BASE + 8 * b + w for w in range(8)]))
        # FEC_GEN_CONSTCOEF=1 (timing probe only, results are garbage): every live field is the
        # case of one fixed coefficient and no coefficient row is read
        constco = bool(os.environ.get("FEC_GEN_CONSTCOEF"))
        fld = (0x53 + 1) * CASE_BYTES

        def const_fields():
            for w in range(ndw if csb < 32 else 4):
                lo = fld if 2 * w < RT else 0
                hi = fld if 2 * w + 1 < RT else 0
                a(f"s_mov_b32 s{S_C[w]}, 0x{(hi << 16) | lo:08x}")
        # the coefficient fields land in the (now free) transpose temporaries under the combos
        if not constco and not early_co:
            a(f"{dsr} {regrange(CO[0], ndw)}, v{COPTR}")
            if csb <= 16:
                a(f"v_add_u32 v{COPTR}, {csb}, v{COPTR}")
        if not os.environ.get("FEC_GEN_PROBE_NOCOMBO"):  # timing probe only (garbage) when set: no combos
            L.extend(combos())
        if AB:
            # QA = s[S_C0:S_C1], QB = s[S_C2:S_C3] (rows of 4 fields: one dword each, the high
            # dwords stay 0); one chain per 8 fields, entered at QA's first field
            assert not constco
            a("s_waitcnt lgkmcnt(0)")
            for w in range(ndw):
                a(f"v_readfirstlane_b32 s{S_C[w if ndw == 4 else 2 * w]}, v{CO[w]}")
            if csb == 32:
                a(f"ds_read_b128 {regrange(CO[0], 4)}, v{COPTR} offset:16")
                a(f"v_add_u32 v{COPTR}, 32, v{COPTR}")
            for ch in range(max(1, RT // 8)):
                if ch:
                    a("s_set_gpr_idx_off")
                    a("s_waitcnt lgkmcnt(0)")
                    for w in range(4):
                        a(f"v_readfirstlane_b32 s{S_C[w]}, v{CO[w]}")
                a(f"s_pack_ll_b32_b16 s{S_TGT}, s{S_C[0]}, s{S_TABHI}")
                a(f"s_lshr_b64 s[{S_C[0]}:{S_C[1]}], s[{S_C[0]}:{S_C[1]}], 16")
                a(f"s_set_gpr_idx_on {acc_base + 64 * ch}, gpr_idx(SRC0,DST)")
                a(f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_TGT}:{S_TGT + 1}]")
        elif constco:
            const_fields()
        else:
            a("s_waitcnt lgkmcnt(0)")
            for w in range(ndw):
                a(f"v_readfirstlane_b32 s{S_C[w]}, v{CO[w]}")
        if csb == 32 and not constco and not AB:  # second half of the offsets lands while the first two chains run
            a(f"ds_read_b128 {regrange(CO[0], 4)}, v{COPTR} offset:16")
            a(f"v_add_u32 v{COPTR}, 32, v{COPTR}")
        # FEC_GEN_INLINE_CASES=c (timing probe only, results are garbage): every chain replaced by the
        # case bodies of the fixed coefficient c, inline on absolute accumulator registers -- no jump,
        # no chain tail, no GPR-index mode: what the case dispatch itself costs
        inline_c = os.environ.get("FEC_GEN_INLINE_CASES")
        if inline_c and not AB:
            L.extend(inline_cases(RT, TL, TH, acc_base, int(inline_c, 0)))
        for ch in range(0 if AB or inline_c else nch):
            if ch == 2:  # RT = 16: offsets 8..15 (no VALU may run in GPR-index mode)
                a("s_set_gpr_idx_off")
                if not constco:
                    a("s_waitcnt lgkmcnt(0)")
                    for w in range(4):
                        a(f"v_readfirstlane_b32 s{S_C[w]}, v{CO[w]}")
            a(f"s_mov_b64 s[{S_CQ}:{S_CQ + 1}], s[{S_C[2 * (ch % 2)]}:{S_C[2 * (ch % 2)] + 1}]")
            a(f"s_pack_ll_b32_b16 s{S_TGT}, s{S_CQ}, s{S_TABHI}")
            if ch % 2 == 0:  # chain 1 continues M0 where chain 0 left it (4 cases later)
                a(f"s_set_gpr_idx_on {acc_base + 32 * ch}, gpr_idx(SRC0,DST)")
            a(f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_TGT}:{S_TGT + 1}]")
        a("s_set_gpr_idx_off")
        a(f"s_sub_u32 s{S_J}, s{S_J}, 1")
        a(f"s_cbranch_scc1 .Lepicall{b}_%=")
        a(f".Lnoepi{b}_%=:")
        a(f"s_sub_u32 s{S_S}, s{S_S}, 1")
        a(f"s_cbranch_scc1 .Lexit_%=")
        ool += [f".Lepicall{b}_%=:", f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_EPI}:{S_EPI + 1}]",
                f"s_sub_u32 s{S_J}, %[k], 1", f"s_branch .Lnoepi{b}_%="]
    a(f"s_branch .Lbody0_%=")
    L.extend(ool)

    # ---- per-block epilogue subroutine ----
    a(".Lepi_%=:")
    if mode == "enc":
        a(f"s_mov_b64 s[{S_O2}:{S_O2 + 1}], s[{S_OUT}:{S_OUT + 1}]")
        a(f"s_mov_b32 s{S_RT}, %[rt]")
    elif epi_pf:
        # the block's row count and first output address are read now and waited for after row 0's
        # transpose; each later address is read one row ahead (into plane registers, dead here)
        a(f"ds_read_b32 v{EPI_RT}, v{OUTPTR} offset:{DEC_REC_RT}")
        a(f"ds_read_b64 v[{EPI_AD}:{EPI_AD + 1}], v{OUTPTR}")
    else:
        a(f"ds_read_b32 v{TMP[2]}, v{OUTPTR} offset:{DEC_REC_RT}")
        a("s_waitcnt lgkmcnt(0)")
        a(f"v_readfirstlane_b32 s{S_RT}, v{TMP[2]}")
    for i in range(RT):
        accs = [acc_base + 8 * i + w for w in range(8)]
        if not (epi_pf and i == 0):
            a(f"s_cmp_le_u32 s{S_RT}, {i}")
            a(f"s_cbranch_scc1 .Lepi_done_%=")
        if T64:
            slots = [accs[SIG[o]] for o in range(8)]  # plane o / word o
            L.extend(transpose64(slots, slots, *t64_scratch(T_BASE)))
        else:
            L.extend(transpose_inplace(accs))
        if epi_pf:
            a(f"v_or3_b32 v{TMP[0]}, v{accs[0]}, v{accs[1]}, v{accs[2]}")
            a(f"v_or3_b32 v{TMP[0]}, v{TMP[0]}, v{accs[3]}, v{accs[4]}")
            a(f"v_or3_b32 v{TMP[0]}, v{TMP[0]}, v{accs[5]}, v{accs[6]}")
            a(f"v_or_b32 v{TMP[0]}, v{TMP[0]}, v{accs[7]}")
            a("s_waitcnt lgkmcnt(0)")  # this row's address (and the last row's flag write)
            if i == 0:  # a block with no rows: row 0's transpose was harmless, nothing is stored
                a(f"v_readfirstlane_b32 s{S_RT}, v{EPI_RT}")
                a(f"s_cmp_le_u32 s{S_RT}, 0")
                a(f"s_cbranch_scc1 .Lepi_done_%=")
            a(f"v_readfirstlane_b32 s{S_O2}, v{EPI_AD}")
            a(f"v_readfirstlane_b32 s{S_O2 + 1}, v{EPI_AD + 1}")
            if i + 1 < RT:
                a(f"ds_read_b64 v[{EPI_AD}:{EPI_AD + 1}], v{OUTPTR} offset:{8 * (i + 1)}")
            a(f"v_cmp_ne_u32 vcc, 0, v{TMP[0]}")
            a(f"v_mov_b32 v{TMP[1]}, 1")
            a("s_and_saveexec_b64 s[{0}:{1}], vcc".format(S_T3, S_T3 + 1))
            a(f"ds_write_b8 v{OUTPTR}, v{TMP[1]} offset:{DEC_REC_NZ + i}")  # non-zero flag (LDS)
            a(f"s_mov_b64 exec, {live}")
        elif mode == "dec":
            a(f"ds_read_b64 v[{TMP[2]}:{TMP[3]}], v{OUTPTR} offset:{8 * i}")
            a(f"v_or3_b32 v{TMP[0]}, v{accs[0]}, v{accs[1]}, v{accs[2]}")
            a(f"v_or3_b32 v{TMP[0]}, v{TMP[0]}, v{accs[3]}, v{accs[4]}")
            a(f"v_or3_b32 v{TMP[0]}, v{TMP[0]}, v{accs[5]}, v{accs[6]}")
            a(f"v_or_b32 v{TMP[0]}, v{TMP[0]}, v{accs[7]}")
            a(f"v_cmp_ne_u32 vcc, 0, v{TMP[0]}")
            a(f"v_mov_b32 v{TMP[1]}, 1")
            a("s_and_saveexec_b64 s[{0}:{1}], vcc".format(S_T3, S_T3 + 1))
            a(f"ds_write_b8 v{OUTPTR}, v{TMP[1]} offset:{DEC_REC_NZ + i}")  # non-zero flag (LDS)
            a(f"s_mov_b64 exec, {live}")
            a("s_waitcnt lgkmcnt(0)")
            a(f"v_readfirstlane_b32 s{S_O2}, v{TMP[2]}")
            a(f"v_readfirstlane_b32 s{S_O2 + 1}, v{TMP[3]}")
        for q in range(NP):
            a(f"s_mov_b64 exec, %[vm{q}]")
            a(f"{st} %[{'so' if sc else 'off'}{q}], {regrange(accs[q * nw], nw)}, s[{S_O2}:{S_O2 + 1}]@STPOL@")
        a(f"s_mov_b64 exec, {live}")
        if mode == "enc":
            a(f"s_add_u32 s{S_O2}, s{S_O2}, %[L]")
            a(f"s_addc_u32 s{S_O2 + 1}, s{S_O2 + 1}, 0")
    a(".Lepi_done_%=:")
    for r in range(acc_base, acc_base + 8 * RT):
        a(f"v_mov_b32 v{r}, 0")
    if mode == "enc":
        a(f"s_add_u32 s{S_OUT}, s{S_OUT}, %[rslo]")  # next block of the group (64-bit step)
        a(f"s_addc_u32 s{S_OUT + 1}, s{S_OUT + 1}, %[rshi]")
    else:
        a(f"v_add_u32 v{OUTPTR}, {DEC_REC_BYTES}, v{OUTPTR}")
    a(f"s_setpc_b64 s[{S_RET}:{S_RET + 1}]")
    a(".Lexit_%=:")
    a("s_waitcnt lgkmcnt(0)")
    a(f"s_mov_b64 exec, s[{S_SAVEEX}:{S_SAVEEX + 1}]")
    a(f"s_mov_b32 m0, s{S_SAVEM0}")
    return L, acc_base + 8 * RT + (4 if touch else 0)


def cstring(lines):
    # cache-policy suffixes of the symbol loads/stores come from FEC_LD_POL / FEC_ST_POL (C string
    # macros, defaults below) so a build can pick them without regenerating
    out = []
    for ln in lines:
        ln = ln.replace("@LDPOL@", '" FEC_LD_POL "').replace("@STPOL@", '" FEC_ST_POL "')
        out.append(f'      "{ln}\\n"')
    return "\n".join(out)


def emit_function(mode, RT, VEC, P, sc=False):
    """sc: the shared-coefficient encode (window blocks, fbn 0): separate per-piece store offsets
    so0.. (a lane's pieces may belong to different windows, whose sources and repairs are laid
    out with different strides)."""
    lines, top = body(mode, RT, VEC, P, sc)
    NP = 32 // VEC
    name = f"bs_{mode}{'sc' if sc else ''}_r{RT}_v{VEC}"
    offs = ", ".join(f"uint32_t off{q}" for q in range(NP))
    if sc:
        offs += ", " + ", ".join(f"uint32_t so{q}" for q in range(NP))
    vms = ", ".join(f"uint64_t vm{q}" for q in range(NP))
    if mode == "enc":
        sig = (f"__device__ __forceinline__ void {name}(uint64_t src, uint64_t rep, uint32_t L, uint32_t rslo, "
               f"uint32_t rshi, uint64_t sdl, uint64_t ll, "
               f"uint32_t nsrc, uint32_t k, uint32_t rt, uint32_t coef, {offs}, {vms})")
        ins = ['[src] "s"(src)', '[rep] "s"(rep)', '[L] "s"(L)', '[rslo] "s"(rslo)', '[rshi] "s"(rshi)', '[sdl] "s"(sdl)', '[ll] "s"(ll)', '[rt] "s"(rt)']
    else:
        sig = (f"__device__ __forceinline__ void {name}(uint32_t intab, uint32_t outtab, uint32_t nsrc, "
               f"uint32_t k, uint32_t coef, {offs}, {vms})")
        ins = ['[intab] "v"(intab)', '[outtab] "v"(outtab)']
    ins += ['[nsrc] "s"(nsrc)', '[k] "s"(k)', '[coef] "v"(coef)']
    ins += [f'[off{q}] "v"(off{q})' for q in range(NP)]
    if sc:
        ins += [f'[so{q}] "v"(so{q})' for q in range(NP)]
    ins += [f'[vm{q}] "s"(vm{q})' for q in range(NP)]
    clob = [f'"v{r}"' for r in range(T_BASE, top)] + [f'"s{r}"' for r in SGPR_CLOBBER] + ['"vcc"', '"scc"', '"memory"']
    out = [sig + " {", "  asm volatile(", cstring(lines), "      :",
           "      : " + ", ".join(ins), "      : " + ", ".join(clob) + ");", "}"]
    return "\n".join(out), top


# ============================================================================ v2: LDS-DMA ring
# The source rows stream into a per-wave LDS ring by LDS-DMA (global_load_lds_dwordx4: one wave-
# instruction moves up to 1 KiB, 16 B per lane, linear in memory and in LDS) issued D-1 sources
# ahead, instead of into D-1 sets of VGPRs.  A step reads its 32 B per lane from the ring straight
# into the plane registers and transposes them in place, so the data costs no VGPRs beyond the
# 8 plane registers: the accumulators and the Four-Russians tables set the occupancy (RT <= 8:
# 4 waves per SIMD instead of 3), and the ring depth only costs LDS.
T2_BASE = int(os.environ.get("FEC_GEN2_BASE", "8"))  # v0 .. v(T2_BASE-1) stay with the compiler
S_PEND, S_PRT, S_COPTR, S_WTAB = 95, 96, 97, 98  # S_WTAB: 98-99
S_INPTR, S_OUTPTR, S_NADDR = 93, 94, 82  # decode only (S_NADDR: 82-83, encode's S_OUT)
SGPR_CLOBBER2 = list(range(60, 100))
CASE_TABLE2 = "fec_bs2_case_table"


def regmap2(mode: str, ntmp: int = 4):
    B = T2_BASE
    assert B % 2 == 0
    tl = {1: B, 2: B + 1, 4: B + 2, 8: B + 3}
    th = {1: B + 4, 2: B + 5, 4: B + 6, 8: B + 7}
    others = [3, 5, 6, 7, 9, 10, 11, 12, 13, 14, 15]
    for i, n in enumerate(others):
        tl[n] = B + 8 + i
        th[n] = B + 19 + i
    tmp = list(range(B + 30, B + 30 + ntmp))
    nxt = B + 30 + ntmp + (ntmp & 1)
    # decode's table pointers and the next row address live in SGPRs (S_INPTR, S_OUTPTR, S_NADDR)
    return {"pl": list(range(B, B + 8)), "tl": tl, "th": th, "tmp": tmp, "acc": nxt}


# bytes per ring slot: a whole column chunk; the unrolled steps address slots by immediates.  FEC_GEN2_SLOT
# (A/B builds only): smaller slots fit more of them in LDS, valid only for chunks that fit a slot
S2_SLOT = int(os.environ.get("FEC_GEN2_SLOT", "2048"))


def body2(mode: str, RT: int, D: int, NDMA: int):
    """One group of blocks x one column chunk, sources through the LDS ring (see above).
    The step is unrolled D times, so step b reads ring slot b and refills slot (b + D - 1) % D with
    immediate offsets (no slot arithmetic).  A step waits for its source's DMAs, issues the reads of
    its 32 B per lane, and only then issues the next DMA (the LDS latency hides under it).
    Wait accounting: vmcnt counts DMAs and stores together in issue order.  At source s's wait the
    younger operations are the NDMA * (D-2) DMAs of sources s+1 .. s+D-2, plus -- during the D-1
    steps after a block's epilogue -- that epilogue's 2 * rt stores; those steps take their wait from
    a table indexed by rt.  Blocks are at least D sources long (the wrapper sizes D <= k), so at most
    one epilogue is ever in the window.  Steps that issue no DMA (the last D-1) wait for everything."""
    NT = int(os.environ.get("FEC_GEN2_NTMP", "2"))
    assert mode == "enc" or NT == 2
    R = regmap2(mode, NT)
    PL, TLm, THm, TMPm = R["pl"], R["tl"], R["th"], R["tmp"]
    XT = [TLm[3], TLm[5], TLm[6], TLm[7]]  # dead until the combos: the forward transpose's temporaries
    acc_base = R["acc"]
    # FEC_GEN2_PROBE_ALIAS=1 (timing probe only, results are garbage): 16-repair encode tiles keep
    # only 8 repairs' accumulators (repairs 8-15 alias 0-7), so the same instruction stream runs at
    # 4 waves/SIMD -- the occupancy a 16-repair tile split over two waves would have
    alias = mode == "enc" and RT == 16 and bool(os.environ.get("FEC_GEN2_PROBE_ALIAS"))
    NACC = 8 if alias else RT
    assert acc_base + 8 * RT <= 256 and acc_base % 2 == 0
    assert D >= 3 and NDMA * (D - 2) + 2 * RT <= 63, "vmcnt is 6 bits"
    assert (D - 1) * S2_SLOT < 65536, "ds_read offsets are 16 bits"
    L = []
    a = L.append
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    a(f"s_mov_b32 s{S_SAVEM0}, m0")
    a(f"s_mov_b64 s[{S_SAVEEX}:{S_SAVEEX + 1}], exec")
    a("s_mov_b64 exec, %[vm0]")  # compute on the lanes that own pieces (the DMAs set their own)
    for i, mk in enumerate(MASKS):
        a(f"s_mov_b32 s{S_MASK[i]}, 0x{mk:08x}")
    a(f"s_getpc_b64 s[{S_TAB}:{S_TAB + 1}]")
    a(f"s_add_u32 s{S_TAB}, s{S_TAB}, {CASE_TABLE2}@rel32@lo+4")
    a(f"s_addc_u32 s{S_TAB + 1}, s{S_TAB + 1}, {CASE_TABLE2}@rel32@hi+12")
    a(f"s_lshr_b32 s{S_TABHI}, s{S_TAB}, 16")
    a(f"s_mov_b32 s{S_TGT + 1}, s{S_TAB + 1}")
    a(f"s_getpc_b64 s[{S_EPI}:{S_EPI + 1}]")
    a(".Lepipc_%=:")
    a(f"s_add_u32 s{S_EPI}, s{S_EPI}, .Lepi_%= - .Lepipc_%=")
    a(f"s_addc_u32 s{S_EPI + 1}, s{S_EPI + 1}, 0")
    a(f"s_getpc_b64 s[{S_WTAB}:{S_WTAB + 1}]")
    a(".Lwtabpc_%=:")
    a(f"s_add_u32 s{S_WTAB}, s{S_WTAB}, .Lwtab_%= - .Lwtabpc_%=")
    a(f"s_addc_u32 s{S_WTAB + 1}, s{S_WTAB + 1}, 0")
    for r in range(acc_base, acc_base + 8 * NACC):
        a(f"v_mov_b32 v{r}, 0")
    a(f"s_mov_b32 s{S_COPTR}, %[coef]")
    if AB:  # QA / QB hold one dword of fields each
        a(f"s_mov_b32 s{S_C[1]}, 0")
        a(f"s_mov_b32 s{S_C[3]}, 0")
    if mode == "enc":
        a(f"s_mov_b64 s[{S_CUR}:{S_CUR + 1}], %[src]")
        a(f"s_mov_b64 s[{S_OUT}:{S_OUT + 1}], %[rep]")
        a(f"s_mov_b32 s{S_JL}, 0")
    else:
        a(f"s_mov_b32 s{S_INPTR}, %[intab]")
        a(f"s_mov_b32 s{S_OUTPTR}, %[outtab]")
    a(f"s_sub_u32 s{S_S}, %[nsrc], 1")
    a(f"s_sub_u32 s{S_J}, %[k], 1")
    a(f"s_sub_u32 s{S_T2}, %[nsrc], {D - 1}")
    a(f"s_cselect_b32 s{S_T2}, 0, s{S_T2}")
    a(f"s_mov_b32 s{S_PEND}, 0")

    T0, T1 = TMPm[0], TMPm[1]

    def naddr_read():
        """decode: issue the read of the next row address (table entry S_INPTR) into T0:T1"""
        return [f"v_mov_b32 v{T1}, s{S_INPTR}",
                f"ds_read_b64 v[{T0}:{T1}], v{T1}",
                f"s_add_u32 s{S_INPTR}, s{S_INPTR}, 8"]

    def naddr_take():
        """decode: the address read by naddr_read (waited for) into S_NADDR"""
        return [f"v_readfirstlane_b32 s{S_NADDR}, v{T0}",
                f"v_readfirstlane_b32 s{S_NADDR + 1}, v{T1}"]

    def dma_issue(slot):
        """DMA of row S_CUR (decode: S_NADDR) into ring slot `slot`"""
        out = []
        if mode == "dec":
            out += [f"s_mov_b64 s[{S_CUR}:{S_CUR + 1}], s[{S_NADDR}:{S_NADDR + 1}]"]
        out += [f"s_add_u32 m0, %[ring], {slot * S2_SLOT}",
                "s_mov_b64 exec, %[vmlo]",  # also the M0 -> LDS-DMA wait state
                f"global_load_lds_dwordx4 %[g1], s[{S_CUR}:{S_CUR + 1}]@LDPOL@"]
        if NDMA == 2:
            out += ["s_add_u32 m0, m0, 1024",
                    "s_mov_b64 exec, %[vmhi]",
                    f"global_load_lds_dwordx4 %[g2], s[{S_CUR}:{S_CUR + 1}]@LDPOL@"]
        out += ["s_mov_b64 exec, %[vm0]"]
        if mode == "enc":  # next row of this block, or the first row of the group's next block
            out += [f"s_add_u32 s{S_JL}, s{S_JL}, 1",
                    f"s_cmp_eq_u32 s{S_JL}, %[k]",
                    f"s_cselect_b64 s[{S_CQ}:{S_CQ + 1}], %[sdl], %[ll]",
                    f"s_cselect_b32 s{S_JL}, 0, s{S_JL}",
                    f"s_add_u32 s{S_CUR}, s{S_CUR}, s{S_CQ}",
                    f"s_addc_u32 s{S_CUR + 1}, s{S_CUR + 1}, s{S_CQ + 1}"]
        return out

    for q in range(D - 1):  # prologue: DMAs for sources 0 .. D-2 into slots 0 .. D-2
        a(f"s_cmp_lt_u32 {q}, %[nsrc]")
        a(f"s_cbranch_scc0 .Lpro_done_%=")
        if mode == "dec":
            L.extend(naddr_read() + ["s_waitcnt lgkmcnt(0)"] + naddr_take() + ["s_nop 4"])
        L.extend(dma_issue(q))
    a(".Lpro_done_%=:")
    if mode == "dec":  # the address of source D-1, taken at step 0
        L.extend(naddr_read())
    csb = coef_row_bytes(RT)
    dsr = "ds_read_b64" if csb == 8 else "ds_read_b128"
    ndw = min(4, csb // 4)
    nch = max(1, RT // 4)
    base_wait = NDMA * (D - 2)
    ool = []
    assert not AB or NT == 2

    def fld_read(ch):
        """AB: chain ch's QA and QB dwords of the coefficient row (FEC_BS_FIELD_SLOT layout) into T0, T1"""
        if csb == 8:
            d0, d1 = 0, 1
        else:
            d0, d1 = 4 * (ch // 2) + ch % 2, 4 * (ch // 2) + 2 + ch % 2
        return [f"v_mov_b32 v{T1}, s{S_COPTR}", f"ds_read2_b32 v[{T0}:{T1}], v{T1} offset0:{d0} offset1:{d1}"]
    const2 = mode == "enc" and NT == 2 and bool(os.environ.get("FEC_GEN2_PROBE_CONST"))

    def data_reads(b):
        return [f"ds_read_b128 v[{PL[0]}:{PL[3]}], %[rd1] offset:{b * S2_SLOT}",
                f"ds_read_b128 v[{PL[4]}:{PL[7]}], %[rd2] offset:{b * S2_SLOT}"]

    for b in range(D):
        a(f".Lstep{b}_%=:")
        a(f"s_sub_u32 s{S_T2}, s{S_T2}, 1")
        a(f"s_cbranch_scc1 .Lnodma{b}_%=")
        a(f"s_cmp_lg_u32 s{S_PEND}, 0")
        a(f"s_cbranch_scc1 .Lbigwait{b}_%=")
        # FEC_GEN2_PROBE_NOVM=1 (timing probe only, results are garbage): no wait for the DMA
        a(f"s_waitcnt vmcnt({63 if os.environ.get('FEC_GEN2_PROBE_NOVM') else base_wait})")
        a(f".Lgot{b}_%=:")
        L.extend(data_reads(b))
        if mode == "dec":  # the address read one step ago (issued before this step's data reads)
            a("s_waitcnt lgkmcnt(2)")
            L.extend(naddr_take())
            a("s_nop 4")  # VALU-written SGPR -> VMEM base
        L.extend(dma_issue((b + D - 1) % D))
        a(f".Lrd{b}_%=:")
        ool += [f".Lnodma{b}_%=:", f"s_mov_b32 s{S_T2}, 0", "s_waitcnt vmcnt(0)"] + data_reads(b) + \
               [f"s_branch .Lrd{b}_%="]
        ool += [f".Lbigwait{b}_%=:",
                f"s_sub_u32 s{S_PEND}, s{S_PEND}, 1",
                f"s_lshl_b32 s{S_CQ}, s{S_PRT}, 3",
                f"s_add_u32 s{S_CQ}, s{S_CQ}, s{S_WTAB}",
                f"s_addc_u32 s{S_CQ + 1}, s{S_WTAB + 1}, 0",
                f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_CQ}:{S_CQ + 1}]",
                f"s_branch .Lgot{b}_%="]
        # the first coefficient fields go out behind the data reads (one wait covers both); decode
        # first waits for the data and issues the next address read (T0:T1 are free again only
        # after the chains), so its fields go out after that read is taken
        if mode == "dec":
            a("s_waitcnt lgkmcnt(0)")
            L.extend(fld_read(0) if AB else [f"v_mov_b32 v{T1}, s{S_COPTR}", f"ds_read_b64 v[{T0}:{T1}], v{T1}"])
        elif AB:
            L.extend(fld_read(0))
            a("s_waitcnt lgkmcnt(1)")
        elif NT >= 4:
            a(f"v_mov_b32 v{TMPm[3]}, s{S_COPTR}")
            a(f"{dsr} {regrange(TMPm[0], ndw)}, v{TMPm[3]}")
            a("s_waitcnt lgkmcnt(1)")
        elif const2:
            a("s_waitcnt lgkmcnt(0)")
        else:
            a(f"v_mov_b32 v{TMPm[1]}, s{S_COPTR}")
            a(f"ds_read_b64 v[{TMPm[0]}:{TMPm[1]}], v{TMPm[1]}")
            # FEC_GEN2_PROBE_NOLDS=1 (timing probe only, results are garbage): no wait for the data reads
            a("s_nop 0" if os.environ.get("FEC_GEN2_PROBE_NOLDS") else "s_waitcnt lgkmcnt(1)")
        if T64:
            L.extend(transpose64([PL[SIG[w]] for w in range(8)], PL, *t64_scratch(T2_BASE)))
        else:
            L.extend(transpose_inplace(PL, XT))
        L.extend(combos(TLm, THm))
        inline2 = os.environ.get("FEC_GEN_INLINE_CASES")  # timing probe only (body(): no dispatch at all)
        if inline2:
            a("s_waitcnt lgkmcnt(0)")
            L.extend(inline_cases(RT, TLm, THm, acc_base, int(inline2, 0)))
            if NT < 4 and not const2:
                a(f"s_add_u32 s{S_COPTR}, s{S_COPTR}, {csb}")
        elif NT >= 4:
            CO = TMPm[:ndw]
            a("s_waitcnt lgkmcnt(0)")
            for w in range(ndw):
                a(f"v_readfirstlane_b32 s{S_C[w]}, v{CO[w]}")
            if csb == 32:
                a(f"v_mov_b32 v{TMPm[3]}, s{S_COPTR}")
                a(f"ds_read_b128 {regrange(CO[0], 4)}, v{TMPm[3]} offset:16")
            a(f"s_add_u32 s{S_COPTR}, s{S_COPTR}, {csb}")
            for ch in range(nch):
                if ch == 2:
                    a("s_set_gpr_idx_off")
                    a("s_waitcnt lgkmcnt(0)")
                    for w in range(4):
                        a(f"v_readfirstlane_b32 s{S_C[w]}, v{CO[w]}")
                a(f"s_mov_b64 s[{S_CQ}:{S_CQ + 1}], s[{S_C[2 * (ch % 2)]}:{S_C[2 * (ch % 2)] + 1}]")
                a(f"s_pack_ll_b32_b16 s{S_TGT}, s{S_CQ}, s{S_TABHI}")
                if ch % 2 == 0:
                    a(f"s_set_gpr_idx_on {acc_base + 32 * (ch % 2 if alias else ch)}, gpr_idx(SRC0,DST)")
                a(f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_TGT}:{S_TGT + 1}]")
        elif const2:
            # FEC_GEN2_PROBE_CONST=1 (timing probe only, results are garbage): the fields are SGPR
            # constants (no LDS reads, no readfirstlane) and GPR-index mode stays on across the chains
            fld = (0x53 + 1) * CASE_BYTES
            a(f"s_set_gpr_idx_on {acc_base}, gpr_idx(SRC0,DST)")
            for ch in range(nch):
                a(f"s_mov_b32 s{S_C[0]}, 0x{(fld << 16) | fld:08x}")
                a(f"s_mov_b32 s{S_C[1]}, 0x{(fld << 16) | fld:08x}")
                a(f"s_mov_b64 s[{S_CQ}:{S_CQ + 1}], s[{S_C[0]}:{S_C[1]}]")
                a(f"s_pack_ll_b32_b16 s{S_TGT}, s{S_CQ}, s{S_TABHI}")
                a(f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_TGT}:{S_TGT + 1}]")
        elif AB:
            # two temporaries: each chain's QA / QB dwords (2 fields each) are read while the previous
            # chain runs; QA and QB are s[S_C0:S_C1] and s[S_C2:S_C3], their high dwords 0
            for ch in range(nch):
                if ch:
                    a("s_set_gpr_idx_off")
                a("s_waitcnt lgkmcnt(0)")
                a(f"v_readfirstlane_b32 s{S_C[0]}, v{T0}")
                a(f"v_readfirstlane_b32 s{S_C[2]}, v{T1}")
                if ch + 1 < nch:
                    L.extend(fld_read(ch + 1))
                a(f"s_pack_ll_b32_b16 s{S_TGT}, s{S_C[0]}, s{S_TABHI}")
                a(f"s_lshr_b64 s[{S_C[0]}:{S_C[1]}], s[{S_C[0]}:{S_C[1]}], 16")
                a(f"s_set_gpr_idx_on {acc_base + 32 * (ch % 2 if alias else ch)}, gpr_idx(SRC0,DST)")
                a(f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_TGT}:{S_TGT + 1}]")
            a(f"s_add_u32 s{S_COPTR}, s{S_COPTR}, {csb}")
        else:
            # two temporaries: each chain's 4 fields (8 B) are read while the previous chain runs
            T0, T1 = TMPm[0], TMPm[1]
            for ch in range(nch):
                if ch:
                    a("s_set_gpr_idx_off")
                a("s_waitcnt lgkmcnt(0)")
                a(f"v_readfirstlane_b32 s{S_C[0]}, v{T0}")
                a(f"v_readfirstlane_b32 s{S_C[1]}, v{T1}")
                if ch + 1 < nch:
                    a(f"v_mov_b32 v{T1}, s{S_COPTR}")
                    a(f"ds_read_b64 v[{T0}:{T1}], v{T1} offset:{8 * (ch + 1)}")
                a(f"s_mov_b64 s[{S_CQ}:{S_CQ + 1}], s[{S_C[0]}:{S_C[1]}]")
                a(f"s_pack_ll_b32_b16 s{S_TGT}, s{S_CQ}, s{S_TABHI}")
                a(f"s_set_gpr_idx_on {acc_base + 32 * (ch % 2 if alias else ch)}, gpr_idx(SRC0,DST)")
                a(f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_TGT}:{S_TGT + 1}]")
            a(f"s_add_u32 s{S_COPTR}, s{S_COPTR}, {csb}")
        a("s_set_gpr_idx_off")
        a(f"s_sub_u32 s{S_J}, s{S_J}, 1")
        a(f"s_cbranch_scc1 .Lepicall{b}_%=")
        a(f".Lnoepi{b}_%=:")
        if mode == "dec":  # the address of source s + D, taken at the next step
            L.extend(naddr_read())
        a(f"s_sub_u32 s{S_S}, s{S_S}, 1")
        a(f"s_cbranch_scc1 .Lexit_%=")
        ool += [f".Lepicall{b}_%=:", f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_EPI}:{S_EPI + 1}]",
                f"s_sub_u32 s{S_J}, %[k], 1", f"s_branch .Lnoepi{b}_%="]
    a(f"s_branch .Lstep0_%=")
    L.extend(ool)
    # the big-wait table: entry i (8 bytes) waits for source s with i repairs' stores in the window
    a(".Lwtab_%=:")
    for i in range(RT + 1):
        a(f"s_waitcnt vmcnt({base_wait + 2 * i})")
        a(f"s_setpc_b64 s[{S_RET}:{S_RET + 1}]")

    # ---- per-block epilogue subroutine: inverse transpose, stores, clear; opens the big-wait window
    a(".Lepi_%=:")
    # decode's scratch: the Four-Russians table registers, dead between a block's last source and
    # the next source's combos (E0:E1 the output address, E2 the record pointer, E3/E4 the flag)
    E = [TLm[3], TLm[5], TLm[6], TLm[7], TLm[9]]
    assert E[0] % 2 == 0 and E[1] == E[0] + 1
    epi_pf = mode == "dec" and DEC_EPI_PF and T64
    assert not epi_pf or set(E).isdisjoint(set(sum(t64_scratch(T2_BASE), [])))
    if mode == "enc":
        a(f"s_mov_b64 s[{S_O2}:{S_O2 + 1}], s[{S_OUT}:{S_OUT + 1}]")
        a(f"s_mov_b32 s{S_RT}, %[rt]")
    elif epi_pf:
        # as the register bodies: the row count and each output address are read a row ahead
        a(f"v_mov_b32 v{E[2]}, s{S_OUTPTR}")
        a(f"ds_read_b32 v{E[3]}, v{E[2]} offset:{DEC_REC_RT}")
        a(f"ds_read_b64 v[{E[0]}:{E[1]}], v{E[2]}")
    else:
        a(f"v_mov_b32 v{E[2]}, s{S_OUTPTR}")
        a(f"ds_read_b32 v{E[0]}, v{E[2]} offset:{DEC_REC_RT}")
        a("s_waitcnt lgkmcnt(0)")
        a(f"v_readfirstlane_b32 s{S_RT}, v{E[0]}")
    for i in range(RT):
        accs = [acc_base + 8 * (i % NACC) + w for w in range(8)]
        if not (epi_pf and i == 0):
            a(f"s_cmp_le_u32 s{S_RT}, {i}")
            a(f"s_cbranch_scc1 .Lepi_done_%=")
        if T64:
            slots = [accs[SIG[o]] for o in range(8)]
            L.extend(transpose64(slots, slots, *t64_scratch(T2_BASE)))
        else:
            L.extend(transpose_inplace(accs, TMPm))
        if epi_pf:
            a("s_waitcnt lgkmcnt(0)")  # this row's address (and the last row's flag write)
            if i == 0:  # a block with no rows: row 0's transpose was harmless, nothing is stored
                a(f"v_readfirstlane_b32 s{S_RT}, v{E[3]}")
                a(f"s_cmp_le_u32 s{S_RT}, 0")
                a(f"s_cbranch_scc1 .Lepi_done_%=")
            a(f"v_readfirstlane_b32 s{S_O2}, v{E[0]}")
            a(f"v_readfirstlane_b32 s{S_O2 + 1}, v{E[1]}")
            if i + 1 < RT:
                a(f"ds_read_b64 v[{E[0]}:{E[1]}], v{E[2]} offset:{8 * (i + 1)}")
            a(f"v_or3_b32 v{E[3]}, v{accs[0]}, v{accs[1]}, v{accs[2]}")
            a(f"v_or3_b32 v{E[3]}, v{E[3]}, v{accs[3]}, v{accs[4]}")
            a(f"v_or3_b32 v{E[3]}, v{E[3]}, v{accs[5]}, v{accs[6]}")
            a(f"v_or_b32 v{E[3]}, v{E[3]}, v{accs[7]}")
            a(f"v_cmp_ne_u32 vcc, 0, v{E[3]}")
            a(f"v_mov_b32 v{E[4]}, 1")
            a("s_and_saveexec_b64 s[{0}:{1}], vcc".format(S_T3, S_T3 + 1))
            a(f"ds_write_b8 v{E[2]}, v{E[4]} offset:{DEC_REC_NZ + i}")
            a("s_mov_b64 exec, %[vm0]")  # 10 instructions after the readfirstlanes: no s_nop
        elif mode == "dec":
            a(f"ds_read_b64 v[{E[0]}:{E[1]}], v{E[2]} offset:{8 * i}")
            a(f"v_or3_b32 v{E[3]}, v{accs[0]}, v{accs[1]}, v{accs[2]}")
            a(f"v_or3_b32 v{E[3]}, v{E[3]}, v{accs[3]}, v{accs[4]}")
            a(f"v_or3_b32 v{E[3]}, v{E[3]}, v{accs[5]}, v{accs[6]}")
            a(f"v_or_b32 v{E[3]}, v{E[3]}, v{accs[7]}")
            a(f"v_cmp_ne_u32 vcc, 0, v{E[3]}")
            a(f"v_mov_b32 v{E[4]}, 1")
            a("s_and_saveexec_b64 s[{0}:{1}], vcc".format(S_T3, S_T3 + 1))
            a(f"ds_write_b8 v{E[2]}, v{E[4]} offset:{DEC_REC_NZ + i}")
            a("s_mov_b64 exec, %[vm0]")
            a("s_waitcnt lgkmcnt(0)")
            a(f"v_readfirstlane_b32 s{S_O2}, v{E[0]}")
            a(f"v_readfirstlane_b32 s{S_O2 + 1}, v{E[1]}")
            a("s_nop 4")  # VALU-written SGPR -> VMEM base
        for q in range(2):
            a(f"s_mov_b64 exec, %[vm{q}]")
            a(f"global_store_dwordx4 %[off{q}], {regrange(accs[4 * q], 4)}, s[{S_O2}:{S_O2 + 1}]@STPOL@")
        a("s_mov_b64 exec, %[vm0]")
        if mode == "enc":
            a(f"s_add_u32 s{S_O2}, s{S_O2}, %[L]")
            a(f"s_addc_u32 s{S_O2 + 1}, s{S_O2 + 1}, 0")
    a(".Lepi_done_%=:")
    a(f"s_mov_b32 s{S_PRT}, s{S_RT}")
    a(f"s_mov_b32 s{S_PEND}, {D - 1}")
    for r in range(acc_base, acc_base + 8 * NACC):
        a(f"v_mov_b32 v{r}, 0")
    if mode == "enc":
        a(f"s_add_u32 s{S_OUT}, s{S_OUT}, %[rslo]")
        a(f"s_addc_u32 s{S_OUT + 1}, s{S_OUT + 1}, %[rshi]")
    else:
        a(f"s_add_u32 s{S_OUTPTR}, s{S_OUTPTR}, {DEC_REC_BYTES}")
    a(f"s_setpc_b64 s[{S_RET}:{S_RET + 1}]")
    a(".Lexit_%=:")
    a("s_waitcnt lgkmcnt(0)")
    a(f"s_mov_b64 exec, s[{S_SAVEEX}:{S_SAVEEX + 1}]")
    a(f"s_mov_b32 m0, s{S_SAVEM0}")
    return L, acc_base + 8 * NACC


def emit_function2(mode, RT, D, NDMA):
    lines, top = body2(mode, RT, D, NDMA)
    name = f"bs2_{mode}_r{RT}_d{NDMA}"
    common = ("uint32_t nsrc, uint32_t k, uint32_t coef, uint32_t ring, "
              "uint32_t g1, uint32_t g2, uint64_t vmlo, uint64_t vmhi, uint32_t rd1, uint32_t rd2, "
              "uint32_t off0, uint32_t off1, uint64_t vm0, uint64_t vm1")
    if mode == "enc":
        sig = (f"__device__ __forceinline__ void {name}(uint64_t src, uint64_t rep, uint32_t L, uint32_t rslo, "
               f"uint32_t rshi, uint64_t sdl, uint64_t ll, uint32_t rt, {common})")
        ins = ['[src] "s"(src)', '[rep] "s"(rep)', '[L] "s"(L)', '[rslo] "s"(rslo)', '[rshi] "s"(rshi)',
               '[sdl] "s"(sdl)', '[ll] "s"(ll)', '[rt] "s"(rt)']
    else:
        sig = f"__device__ __forceinline__ void {name}(uint32_t intab, uint32_t outtab, {common})"
        ins = ['[intab] "s"(intab)', '[outtab] "s"(outtab)']
    ins += ['[nsrc] "s"(nsrc)', '[k] "s"(k)', '[coef] "s"(coef)', '[ring] "s"(ring)', '[g1] "v"(g1)', '[g2] "v"(g2)', '[vmlo] "s"(vmlo)', '[vmhi] "s"(vmhi)',
            '[rd1] "v"(rd1)', '[rd2] "v"(rd2)', '[off0] "v"(off0)', '[off1] "v"(off1)', '[vm0] "s"(vm0)',
            '[vm1] "s"(vm1)']
    clob = [f'"v{r}"' for r in range(T2_BASE, top)] + [f'"s{r}"' for r in SGPR_CLOBBER2] + ['"vcc"', '"scc"',
                                                                                          '"memory"']
    out = [sig + " {", "  asm volatile(", cstring(lines), "      :",
           "      : " + ", ".join(ins), "      : " + ", ".join(clob) + ");", "}"]
    return "\n".join(out), top


RING_DEPTH = {("enc", 1): 4, ("enc", 2): 4, ("enc", 4): 4, ("enc", 8): 4, ("enc", 16): 4,
              ("dec", 1): 4, ("dec", 2): 4, ("dec", 4): 4, ("dec", 8): 4, ("dec", 16): 5}


def ring_depth(mode: str, RT: int) -> int:
    return int(os.environ.get(f"FEC_GEN2_D_{mode.upper()}_RT{RT}") or os.environ.get("FEC_GEN2_D")
               or RING_DEPTH[(mode, RT)])


DEC_REC_BYTES = 160  # per-block decode record in LDS: 16 x 8 B output addresses | rt @136 | nz flags @144
DEC_REC_RT = 136
DEC_REC_NZ = 144


def data_base(mode: str) -> int:
    return DATA_BASE if mode == "enc" else NADDR + 2  # tuples must start on an even VGPR


def prefetch_depth(mode: str, RT: int, VEC: int = 16) -> int:
    """Register prefetch depth P (source rows in flight per wave).  Prefer 3 waves/SIMD
    (<= 168 VGPRs) when that still leaves P >= PMIN3 (4 for encode, 2 for decode); otherwise
    take everything up to 256 VGPRs at 2 waves/SIMD.  Bounded by the 6-bit vmcnt: NP * (P - 1) <= 63.
    The recover kernels run one group per workgroup (no grid-stride loop), so the compiler keeps
    nothing live across the asm beyond v0-v31 and the decode budgets need no margin (round 2 carried
    14 VGPRs of loop invariants; -Rpass-analysis=kernel-resource-usage, profiles/r03_kernel_resources.txt)."""
    NP = 32 // VEC
    margin = int(os.environ.get("FEC_GEN_DEC_MARGIN", "0")) if mode == "dec" else 0
    budget3 = int(os.environ.get("FEC_GEN_VGPR3", "168")) - margin
    # 2-wave budget for decode: RT=8 needs a larger margin than RT=16 (measured: a 242 budget at
    # RT=8 compiled to 256 VGPRs + 4 AGPRs = 1 wave/SIMD, k32 e8 apply 13 ms -> 7.6 ms at 222)
    budget2 = 256 - margin - (8 if mode == "dec" and RT <= 8 else 0)
    tv = 4 if TOUCH and mode == "dec" and EARLY_PF else 0
    fits = lambda P, lim: data_base(mode) + 8 * P + 8 * RT + tv <= lim and NP * (P - (0 if EARLY_PF else 1)) <= 63 \
        and (not tv or (NP + 1) * (P - 1) + 1 <= 63)
    # 4-unknown decode tiles take the 2-wave budget: 19 rows in flight at 2 waves/SIMD streamed the k16 e4
    # apply 2.3 % faster than 8 at 3 waves (profiles/r03_ab_dec_occupancy.log); 8-unknown tiles keep 3
    # waves (2 waves: +13-20 %)
    forced = os.environ.get(f"FEC_GEN_LIMIT_{mode.upper()}_RT{RT}") or os.environ.get(f"FEC_GEN_LIMIT_RT{RT}") or \
        ("256" if mode == "dec" and RT == 4 else None)
    if forced:  # A/B: VGPR limit for this tile size
        return max([P for P in range(2, 33) if fits(P, int(forced) - margin)] or [2])
    p3 = max([P for P in range(2, 33) if fits(P, budget3)] or [0])
    # decode takes 3 waves/SIMD even at P = 2: RT=8 at 3 waves and P=2 ran 14.7 % faster than at 2
    # waves and P=12 (profiles/r01_ab_prefetch.log); encode keeps P >= 4 (its RT=8 tile fits P=4)
    pmin3 = int(os.environ.get("FEC_GEN_PMIN3", "2" if mode == "dec" else "4"))
    if p3 >= pmin3:
        return min(p3, int(os.environ.get("FEC_GEN_PMAX", "8")))
    return max([P for P in range(2, 33) if fits(P, budget2)] or [2])


CONFIGS = [(RT, VEC) for VEC in (16, 8, 4) for RT in (1, 2, 4, 8, 16)]


_V1_LAYOUT_NAMES = ("T_BASE", "TL", "TH", "TMP", "CO", "COPTR", "INPTR", "OUTPTR", "NADDR", "DATA_BASE", "XS",
                    "PL", "V1_TABLE")


def v1_compact_layout():
    """The register-prefetch bodies on the ring bodies' compact register map (table registers from
    v8, the ring case table): 8-repair encode tiles then fit 4 waves/SIMD (128 VGPRs) at a prefetch
    depth of 2 -- k32 r8 encode -1.8 % against 3 waves at depth 4 (profiles/r02_ab_v1_compact.log)."""
    R = regmap2("enc", 4)
    coptr = T2_BASE + 34
    tl, th = R["tl"], R["th"]
    return {"T_BASE": T2_BASE, "TL": tl, "TH": th, "TMP": R["tmp"], "CO": R["tmp"], "COPTR": coptr,
            "INPTR": coptr + 1, "OUTPTR": coptr + 2, "NADDR": coptr + 4,
            "DATA_BASE": coptr + 1 + ((coptr + 1) & 1),
            "XS": [tl[3], tl[5], tl[6], tl[7], th[3], th[5], th[6], th[7]],
            "PL": [tl[1], tl[2], tl[4], tl[8], th[1], th[2], th[4], th[8]], "V1_TABLE": CASE_TABLE2}


class _Layout:
    """Temporarily switch the module's v1 register map (the v1 emitters read the globals)."""

    def __init__(self, m):
        self.m = m

    def __enter__(self):
        g = globals()
        self.saved = {n: g[n] for n in _V1_LAYOUT_NAMES}
        if self.m:
            g.update(self.m)

    def __exit__(self, *exc):
        globals().update(self.saved)


# encode tile sizes whose register-prefetch bodies use the compact map at 4 waves/SIMD
COMPACT_ENC = {int(x) for x in os.environ.get("FEC_GEN_COMPACT_ENC", "8").split(",") if x}
COMPACT_DEC = {int(x) for x in os.environ.get("FEC_GEN_COMPACT_DEC", "").split(",") if x}
COMPACT_VGPRS = 128


def compact_vgprs(RT: int) -> int:
    """VGPR budget of a compact-map encode tile (512 / budget = waves per SIMD)."""
    return int(os.environ.get(f"FEC_GEN_COMPACT_VGPRS_RT{RT}") or COMPACT_VGPRS)


def main():
    selfcheck()
    selfcheck_t64()
    parts = ["// GENERATED by pquic_amd/csrc/gen_bitslice.py -- do not edit.",
             "// Bitsliced GF(2^8) multiply-accumulate bodies for gfx950 (see the generator's docstring).",
             "#pragma once",
             "#include <hip/hip_runtime.h>",
             "#include <stdint.h>",
             "",
             f"#define FEC_BS_CASE_BYTES {CASE_BYTES}",
             "// LDS coefficient row per source: max(4, RT) u16 fields (c + 1) * FEC_BS_CASE_BYTES, 0 ends a chain",
             "#define FEC_BS_COEF_ROW_BYTES(RT) (2 * ((RT) < 4 ? 4 : (RT)))",
             f"#define FEC_BS_AB {int(AB)}  // two case tables (even / odd chain positions, gen_bitslice.py AB)",
             f"#define FEC_BS_TABLE_B {TABLE_B}",
             "// slot of repair (unknown) i in its row and its field for coefficient c: with AB, each group of",
             "// g = 8 (RT >= 8) or 4 fields holds the even positions' fields (queue QA) before the odd ones'",
             "// (queue QB), and odd positions point into table B",
             "#if FEC_BS_AB",
             "#define FEC_BS_FIELD_SLOT(RT, i) ((((RT) >= 8 ? 8 : 4) * ((i) / ((RT) >= 8 ? 8 : 4))) + \\",
             "    (((i) & 1) ? ((RT) >= 8 ? 4 : 2) : 0) + ((i) % ((RT) >= 8 ? 8 : 4)) / 2)",
             "#define FEC_BS_FIELD(c, i) ((uint16_t)(((c) + 1u) * FEC_BS_CASE_BYTES + (((i) & 1) ? FEC_BS_TABLE_B : 0)))",
             "#else",
             "#define FEC_BS_FIELD_SLOT(RT, i) (i)",
             "#define FEC_BS_FIELD(c, i) ((uint16_t)(((c) + 1u) * FEC_BS_CASE_BYTES))",
             "#endif",
             "#ifndef FEC_LD_POL",
             "// symbol loads non-temporal: k16 r4 encode -5.3 %, decode -1.3 %, k32 e8 decode -1.7 %, k64 r16",
             "// L9000 encode / decode -1.2 % (profiles/r04_ab_ld_policy.log)",
             "#define FEC_LD_POL \" nt\"",
             "#endif",
             "#ifndef FEC_LD_POL_SC",
             "// the shared-coefficient window bodies keep the default policy: overlapping windows read each",
             "// source row k / step times, the repeats from L2 (nt: k32 r8 step 8 14.96 -> 19.30 ms)",
             "#define FEC_LD_POL_SC \"\"",
             "#endif",
             "#ifndef FEC_LD_POL_COMPACT",
             "// the compact-map bodies (8-repair encode tiles) keep the default policy: nt loads leave the k32 r8",
             "// encode's time unchanged (+0.1 %, profiles/r04_ab_ld_policy2.log) and raise its HBM reads from",
             "// 1.004x to 1.032x the algorithmic bytes (profiles/r04_pmc_nt.json)",
             "#define FEC_LD_POL_COMPACT \"\"",
             "#endif",
             "#ifndef FEC_ST_POL",
             "#define FEC_ST_POL \" nt\"  // repair / recovered symbol stores",
             "#endif",
             "",
             "// Shared 256-case table: case c applies  acc[v0..v7] ^= TL[.] ^ TH[.]  for coefficient c.",
             "// It lives in the body of a never-launched kernel (HIP drops module-level asm in the",
             "// device pass); the data-path bodies reach it through a PC-relative relocation.",
             "__global__ void fec_bs_case_table_holder() {",
             "  asm volatile(",
             '    "s_endpgm\\n"']
    parts += [f'    "{ln}\\n"' for ln in emit_table()]
    parts += ['    "  s_endpgm\\n");', "}", ""]
    # the LDS-ring bodies' table: the same cases over their plane-register numbering (regmap2)
    R2 = regmap2("enc")
    parts += ["// The same 256 cases over the LDS-ring bodies' plane registers (regmap2).",
              "__global__ void fec_bs2_case_table_holder() {",
              "  asm volatile(",
              '    "s_endpgm\\n"']
    parts += [f'    "{ln}\\n"' for ln in emit_table(CASE_TABLE2, R2["tl"], R2["th"])]
    parts += ['    "  s_endpgm\\n");', "}", ""]
    parts += ["// The tables' runtime addresses (the case tails build targets as TAB.hi:TAB.lo[31:16]:offset,",
              "// which needs 64 KiB alignment): the engine checks them once per device before any launch.",
              "__global__ void fec_bs_case_table_addr(uint64_t *out) {",
              "  uint32_t lo, hi, lo2, hi2;",
              "  asm volatile(",
              '    "s_getpc_b64 s[60:61]\\n"',
              '    "s_add_u32 s60, s60, fec_bs_case_table@rel32@lo+4\\n"',
              '    "s_addc_u32 s61, s61, fec_bs_case_table@rel32@hi+12\\n"',
              '    "s_mov_b32 %0, s60\\n"',
              '    "s_mov_b32 %1, s61\\n"',
              '    "s_getpc_b64 s[60:61]\\n"',
              f'    "s_add_u32 s60, s60, {CASE_TABLE2}@rel32@lo+4\\n"',
              f'    "s_addc_u32 s61, s61, {CASE_TABLE2}@rel32@hi+12\\n"',
              '    "s_mov_b32 %2, s60\\n"',
              '    "s_mov_b32 %3, s61\\n"',
              '    : "=s"(lo), "=s"(hi), "=s"(lo2), "=s"(hi2) : : "s60", "s61");',
              "  if (threadIdx.x == 0) {",
              "    out[0] = ((uint64_t)hi << 32) | lo;",
              "    out[1] = ((uint64_t)hi2 << 32) | lo2;",
              "  }",
              "}", ""]
    tops = {}
    for RT in sorted(COMPACT_ENC):
        parts.append(f"#define FEC_V1_ENC{RT}_WAVES {512 // compact_vgprs(RT)}  // compact-map encode tiles (v1_compact_layout)")
    for RT in sorted(COMPACT_DEC):
        parts.append(f"#define FEC_V1_DEC{RT}_WAVES {512 // compact_vgprs(RT)}  // compact-map decode tiles")
    for mode in ("enc", "dec"):
        for RT, VEC in CONFIGS:
            compact = RT in (COMPACT_ENC if mode == "enc" else COMPACT_DEC)
            with _Layout(v1_compact_layout() if compact else None):
                if compact:
                    NP = 32 // VEC
                    margin = int(os.environ.get("FEC_GEN_DEC_MARGIN", "14")) if mode == "dec" else 0
                    P = max(P for P in range(2, 33) if data_base(mode) + 8 * P + 8 * RT <= compact_vgprs(RT) - margin
                            and NP * (P - (0 if EARLY_PF else 1)) <= 63)
                else:
                    P = prefetch_depth(mode, RT, VEC)
                fn, top = emit_function(mode, RT, VEC, P)
                if compact:  # the compact-map bodies' loads take their own policy macro (A/B builds)
                    fn = fn.replace('" FEC_LD_POL "', '" FEC_LD_POL_COMPACT "')
            tops[(mode, RT, VEC, P)] = top
            parts.append(fn)
            parts.append("")
    # shared-coefficient encode bodies (window blocks): wide register map, 16-B pieces
    for RT in (1, 2, 4, 8):
        P = prefetch_depth("enc", RT, 16)
        fn, top = emit_function("enc", RT, 16, P, sc=True)
        fn = fn.replace('" FEC_LD_POL "', '" FEC_LD_POL_SC "')  # overlapping windows re-read rows from L2
        tops[("encsc", RT, 16, P)] = top
        parts.append(fn)
        parts.append("")
    parts.append(f"#define FEC_BS2_BASE {T2_BASE}")
    parts.append(f"#define FEC_BS2_RT16_WAVES {4 if os.environ.get('FEC_GEN2_PROBE_ALIAS') else 3}  // 16-repair ring encode waves/SIMD")
    parts.append(f"#define FEC_BS2_SLOT {S2_SLOT}  // ring slot bytes (the bodies address slots by immediates)")
    # the ring bodies ship for 16-repair / 16-unknown tiles only (round 2's A/Bs retired them for
    # smaller tiles: k32 r8 +2 %, decode +10-20 %); FEC_GEN2_TILES=1,2,4,8,16 emits the rest for A/B builds
    tiles2 = [int(x) for x in os.environ.get("FEC_GEN2_TILES", "16").split(",") if x]
    for mode in ("enc", "dec"):
        for RT in tiles2:
            D = ring_depth(mode, RT)
            parts.append(f"#define FEC_BS2_D_{mode.upper()}_RT{RT} {D}")
            for NDMA in (1, 2):
                fn, top = emit_function2(mode, RT, D, NDMA)
                tops[(mode + "2", RT, NDMA, D)] = top
                parts.append(fn)
                parts.append("")
    with open(OUT, "w") as f:
        f.write("\n".join(parts))
    print(f"wrote {OUT}: {len(CONFIGS) * 2} + 4 + {4 * len(tiles2)} bodies, max VGPR {max(tops.values())}")


if __name__ == "__main__":
    main()
