"""oracle/oracle_py.py -- TEST INFRASTRUCTURE ONLY.

ctypes bindings for the CPU restatement (oracle/liboracle.so) and, in the survey
container only, the natively compiled reference (oracle/_ref/libfecref.so).
Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; never by
the product package.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libfecref.so")

DEC_RECOVERED, DEC_NOTHING, DEC_REF_UB = 0, 1, 2

_u8p = C.POINTER(C.c_uint8)
_u16p = C.POINTER(C.c_uint16)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)


def _ptr(a: np.ndarray, t=_u8p):
    return a.ctypes.data_as(t)


def synth_bytes(nbytes: int, seed: int, offset: int = 0) -> np.ndarray:
    """Counter-based SplitMix64 bytes (same stream as oracle_synth_fill / the device fill)."""
    first = offset >> 3
    last = (offset + nbytes + 7) >> 3
    idx = np.arange(first, last + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (idx + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    b = z.astype("<u8").view(np.uint8)
    s = offset - (first << 3)
    return b[s:s + nbytes].copy()


class Oracle:
    def __init__(self, path: str = LIB_PATH):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        L = C.CDLL(path)
        self.lib = L
        L.oracle_gf_tables.argtypes = [_u8p, _u8p]
        L.oracle_gf_mul.argtypes = [C.c_uint8, C.c_uint8]
        L.oracle_gf_mul.restype = C.c_uint8
        L.oracle_tinymt32_first.argtypes = [C.c_uint32]
        L.oracle_tinymt32_first.restype = C.c_uint32
        L.oracle_tinymt32_stream.argtypes = [C.c_uint32, C.c_int, _u32p]
        L.oracle_rlc_coefs.argtypes = [C.c_uint32, C.c_int, _u8p]
        L.oracle_rlc_seed.argtypes = [C.c_uint32, C.c_uint32]
        L.oracle_rlc_seed.restype = C.c_uint32
        pp = C.POINTER(_u8p)
        L.oracle_rlc_encode_block.argtypes = [C.c_uint32, C.c_int, C.c_int, pp, _u16p, pp, _u16p]
        L.oracle_xor_encode_block.argtypes = [C.c_int, C.c_int, pp, _u16p, _u8p, _u16p]
        L.oracle_rlc_decode_block.argtypes = [C.c_uint32, C.c_int, C.c_int, pp, _u16p, pp, _u16p,
                                              _u32p, pp, _u16p, _u8p]
        L.oracle_xor_decode_block.argtypes = [C.c_int, C.c_int, pp, _u16p, pp, _u16p, _u8p, _u16p,
                                              C.POINTER(C.c_int)]
        L.oracle_rlc_encode_batch.argtypes = [_u8p, _u8p, C.c_uint64, C.c_int, C.c_int, C.c_int,
                                              C.c_uint32, C.c_int]
        L.oracle_rlc_decode_batch.argtypes = [_u8p, _u8p, C.c_uint64, C.c_int, C.c_int, C.c_int,
                                              C.c_uint32, _u64p, _u64p, _u8p, _u64p, C.c_int]
        L.oracle_xor_encode_batch.argtypes = [_u8p, _u8p, C.c_uint64, C.c_int, C.c_int, C.c_int]
        L.oracle_xor_decode_batch.argtypes = [_u8p, _u8p, C.c_uint64, C.c_int, C.c_int, _u64p, _u64p,
                                              _u8p, _u64p, C.c_int]
        L.oracle_synth_fill.argtypes = [_u8p, C.c_uint64, C.c_uint64, C.c_uint64]
        L.oracle_cpu_count.restype = C.c_int

    # ---- scalar helpers ----
    def gf_tables(self):
        mul = np.zeros((256, 256), np.uint8)
        inv = np.zeros(256, np.uint8)
        self.lib.oracle_gf_tables(_ptr(mul), _ptr(inv))
        return mul, inv

    def tinymt32(self, seed: int, n: int) -> np.ndarray:
        out = np.zeros(n, np.uint32)
        self.lib.oracle_tinymt32_stream(seed, n, _ptr(out, _u32p))
        return out

    def coefs(self, seed: int, n: int) -> np.ndarray:
        out = np.zeros(n, np.uint8)
        self.lib.oracle_rlc_coefs(seed, n, _ptr(out))
        return out

    def seed(self, fbn: int, i: int) -> int:
        return int(self.lib.oracle_rlc_seed(fbn, i))

    def cpu_count(self) -> int:
        return int(self.lib.oracle_cpu_count())

    # ---- per-block, variable-length ----
    def rlc_encode_block(self, fbn: int, srcs: list, r: int):
        k = len(srcs)
        keep = [np.ascontiguousarray(s, np.uint8) for s in srcs]
        lens = np.array([len(s) for s in keep], np.uint16)
        maxl = int(lens.max()) if k else 0
        reps = [np.zeros(max(maxl, 1), np.uint8) for _ in range(r)]
        sp = (_u8p * k)(*[_ptr(s) for s in keep])
        rp = (_u8p * max(r, 1))(*[_ptr(x) for x in reps])
        rl = np.zeros(max(r, 1), np.uint16)
        ret = self.lib.oracle_rlc_encode_block(fbn, k, r, sp, _ptr(lens, _u16p), rp, _ptr(rl, _u16p))
        return ret, [reps[i][: rl[i]].copy() for i in range(r)] if ret == 0 else []

    def xor_encode_block(self, srcs: list):
        k = len(srcs)
        keep = [np.ascontiguousarray(s, np.uint8) for s in srcs]
        lens = np.array([len(s) for s in keep], np.uint16)
        rep = np.zeros(max(int(lens.max()), 1), np.uint8)
        rl = np.zeros(1, np.uint16)
        sp = (_u8p * k)(*[_ptr(s) for s in keep])
        ret = self.lib.oracle_xor_encode_block(k, 1, sp, _ptr(lens, _u16p), _ptr(rep), _ptr(rl, _u16p))
        return ret, rep[: rl[0]].copy()

    def rlc_decode_block(self, fbn: int, srcs: list, reps: list, rep_seeds=None):
        """srcs/reps: lists with None for missing symbols. Returns (status, {j: bytes})."""
        k, r = len(srcs), len(reps)
        ks = [None if s is None else np.ascontiguousarray(s, np.uint8) for s in srcs]
        kr = [None if s is None else np.ascontiguousarray(s, np.uint8) for s in reps]
        sl = np.array([0 if s is None else len(s) for s in ks], np.uint16)
        rl = np.array([0 if s is None else len(s) for s in kr], np.uint16)
        maxl = max([len(s) for s in kr if s is not None] + [1])
        outs = [np.zeros(max(maxl, 65535), np.uint8) for _ in range(k)]
        sp = (_u8p * k)(*[None if s is None else _ptr(s) for s in ks])
        rp = (_u8p * max(r, 1))(*[None if s is None else _ptr(s) for s in kr])
        op = (_u8p * k)(*[_ptr(o) for o in outs])
        ol = np.zeros(k, np.uint16)
        rec = np.zeros(k, np.uint8)
        seeds = None if rep_seeds is None else np.asarray(rep_seeds, np.uint32)
        st = self.lib.oracle_rlc_decode_block(fbn, k, r, sp, _ptr(sl, _u16p), rp, _ptr(rl, _u16p),
                                              None if seeds is None else _ptr(seeds, _u32p),
                                              op, _ptr(ol, _u16p), _ptr(rec))
        return st, {j: outs[j][: ol[j]].copy() for j in range(k) if rec[j]}

    def xor_decode_block(self, srcs: list, reps: list):
        k, r = len(srcs), len(reps)
        ks = [None if s is None else np.ascontiguousarray(s, np.uint8) for s in srcs]
        kr = [None if s is None else np.ascontiguousarray(s, np.uint8) for s in reps]
        sl = np.array([0 if s is None else len(s) for s in ks], np.uint16)
        rl = np.array([0 if s is None else len(s) for s in kr], np.uint16)
        out = np.zeros(65536, np.uint8)
        ol = np.zeros(1, np.uint16)
        idx = C.c_int(-1)
        sp = (_u8p * k)(*[None if s is None else _ptr(s) for s in ks])
        rp = (_u8p * max(r, 1))(*[None if s is None else _ptr(s) for s in kr])
        st = self.lib.oracle_xor_decode_block(k, r, sp, _ptr(sl, _u16p), rp, _ptr(rl, _u16p),
                                              _ptr(out), _ptr(ol, _u16p), C.byref(idx))
        return st, ({idx.value: out[: ol[0]].copy()} if st == DEC_RECOVERED else {})

    # ---- batched, fixed layout ----
    def rlc_encode_batch(self, src: np.ndarray, r: int, fbn_base: int = 0, nthreads: int = 0):
        nb, k, L = src.shape
        rep = np.zeros((nb, r, L), np.uint8)
        self.lib.oracle_rlc_encode_batch(_ptr(src), _ptr(rep), nb, k, r, L, fbn_base, nthreads)
        return rep

    def rlc_decode_batch(self, src: np.ndarray, rep: np.ndarray, src_present: np.ndarray,
                         rep_present: np.ndarray, fbn_base: int = 0, nthreads: int = 0):
        """src is updated in place with recovered symbols. Returns (status, recovered_mask)."""
        nb, k, L = src.shape
        r = rep.shape[1]
        st = np.zeros(nb, np.uint8)
        rec = np.zeros((nb, 2), np.uint64)
        self.lib.oracle_rlc_decode_batch(_ptr(src), _ptr(rep), nb, k, r, L, fbn_base,
                                         _ptr(src_present, _u64p), _ptr(rep_present, _u64p),
                                         _ptr(st), _ptr(rec, _u64p), nthreads)
        return st, rec

    def xor_encode_batch(self, src: np.ndarray, nthreads: int = 0):
        nb, k, L = src.shape
        rep = np.zeros((nb, 1, L), np.uint8)
        self.lib.oracle_xor_encode_batch(_ptr(src), _ptr(rep), nb, k, L, nthreads)
        return rep

    def xor_decode_batch(self, src, rep, src_present, rep_present, nthreads: int = 0):
        nb, k, L = src.shape
        st = np.zeros(nb, np.uint8)
        rec = np.zeros((nb, 2), np.uint64)
        self.lib.oracle_xor_decode_batch(_ptr(src), _ptr(rep), nb, k, L, _ptr(src_present, _u64p),
                                         _ptr(rep_present, _u64p), _ptr(st), _ptr(rec, _u64p),
                                         nthreads)
        return st, rec


class Reference:
    """The reference's own scheme pluglets, compiled natively (survey container only)."""

    def __init__(self, path: str = REF_PATH):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        L = C.CDLL(path)
        self.lib = L
        L.ref_gf_tables.argtypes = [_u8p, _u8p]
        L.ref_create_outputs.argtypes = [C.c_int, _u64p, _u64p]
        L.ref_tinymt32.argtypes = [C.c_uint32, C.c_int, _u32p]
        L.ref_encode.argtypes = [C.c_int, C.c_uint32, C.c_int, C.c_int, _u8p, _u16p, C.c_int, _u8p,
                                 C.c_int, _u64p, _u16p]
        L.ref_decode.argtypes = [C.c_int, C.c_uint32, C.c_int, C.c_int, _u8p, _u16p, _u8p, C.c_int,
                                 _u8p, _u16p, _u8p, _u64p, C.c_int, _u8p, _u16p, _u8p, C.c_int, _u32p]
        L.ref_rlc_encode_batch.argtypes = [_u8p, _u8p, C.c_uint64, C.c_int, C.c_int, C.c_int,
                                           C.c_uint32]
        L.ref_layout.argtypes = [_u64p]

    def gf_tables(self):
        mul = np.zeros((256, 256), np.uint8)
        inv = np.zeros(256, np.uint8)
        assert self.lib.ref_gf_tables(_ptr(mul), _ptr(inv)) == 0
        return mul, inv

    def tinymt32(self, seed: int, n: int):
        out = np.zeros(n, np.uint32)
        self.lib.ref_tinymt32(seed, n, _ptr(out, _u32p))
        return out

    def layout(self):
        out = np.zeros(8, np.uint64)
        self.lib.ref_layout(_ptr(out, _u64p))
        return [int(x) for x in out]

    def encode_block(self, xor: bool, fbn: int, srcs: list, r: int):
        k = len(srcs)
        maxl = max(len(s) for s in srcs)
        stride = max(maxl, 1)
        buf = np.zeros((k, stride), np.uint8)
        lens = np.zeros(k, np.uint16)
        for j, s in enumerate(srcs):
            buf[j, : len(s)] = s
            lens[j] = len(s)
        rep = np.zeros((max(r, 1), stride), np.uint8)
        fp = np.zeros(max(r, 1), np.uint64)
        rl = np.zeros(max(r, 1), np.uint16)
        ret = self.lib.ref_encode(int(xor), fbn, k, r, _ptr(buf), _ptr(lens, _u16p), stride,
                                  _ptr(rep), stride, _ptr(fp, _u64p), _ptr(rl, _u16p))
        return ret, [rep[i, : rl[i]].copy() for i in range(r)], [int(x) for x in fp[:r]]

    def decode_block(self, xor: bool, fbn: int, srcs: list, reps: list, rep_fpids: list,
                     with_fpids: bool = False):
        """Returns (ret, {j: bytes}) or, with_fpids, (ret, {j: bytes}, {j: recovered source FPID})."""
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
        fp[:r] = rep_fpids
        out = np.zeros((k, stride), np.uint8)
        ol = np.zeros(k, np.uint16)
        rec = np.zeros(k, np.uint8)
        ofp = np.zeros(k, np.uint32)
        ret = self.lib.ref_decode(int(xor), fbn, k, r, _ptr(sb), _ptr(sl, _u16p), _ptr(spres), stride,
                                  _ptr(rb), _ptr(rl, _u16p), _ptr(rpres), _ptr(fp, _u64p), stride,
                                  _ptr(out), _ptr(ol, _u16p), _ptr(rec), stride, _ptr(ofp, _u32p))
        got = {j: out[j, : ol[j]].copy() for j in range(k) if rec[j]}
        if with_fpids:
            return ret, got, {j: int(ofp[j]) for j in range(k) if rec[j]}
        return ret, got

    def rlc_encode_batch(self, src: np.ndarray, r: int, fbn_base: int = 0):
        nb, k, L = src.shape
        rep = np.zeros((nb, r, L), np.uint8)
        assert self.lib.ref_rlc_encode_batch(_ptr(src), _ptr(rep), nb, k, r, L, fbn_base) == 0
        return rep
