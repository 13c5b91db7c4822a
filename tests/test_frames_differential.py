"""Frame codecs against the reference's own frame code, live, on many more random inputs than the
committed fixtures (tests/golden/frames.json holds about 1100 cases from one seed): the same
generators as tests/golden/gen_frames.py, other seeds, and each case checked against
oracle/_ref/libfecref.so (the reference's fec.h helpers and frame pluglets, built by
`make -C oracle ref` from /root/reference; the test skips where that build is absent, e.g. on the GPU
boxes).  Pure host C, CPU suite."""
import ctypes as C
import os
import random
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
REF = os.path.join(ROOT, "oracle", "_ref", "libfecref.so")
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import test_frames  # noqa: E402
from test_frames import SKIP_FN, Hdr, synthetic_skip  # noqa: E402

N = int(os.environ.get("PQUIC_FRAMES_FUZZ_CASES", "3000"))


@pytest.fixture(scope="module")
def ref():
    if not os.path.exists(REF):
        pytest.skip("reference build oracle/_ref/libfecref.so absent")
    import gen_frames
    return gen_frames.lib()


@pytest.fixture(scope="module")
def lib():
    """the engine library with test_frames' bindings"""
    if not os.path.exists(test_frames.LIB):
        pytest.skip("engine library not built")
    L = C.CDLL(test_frames.LIB)
    u8p = C.POINTER(C.c_uint8)
    L.pquic_fec_write_fec_frame_header.argtypes = [C.POINTER(Hdr), u8p]
    L.pquic_fec_write_fec_frame_header.restype = C.c_size_t
    L.pquic_fec_parse_fec_frame_header.argtypes = [u8p, C.POINTER(Hdr)]
    L.pquic_fec_write_sfpid_frame.argtypes = [C.c_uint32, u8p, C.c_size_t, C.POINTER(C.c_size_t)]
    L.pquic_fec_parse_sfpid_frame.argtypes = [u8p]
    L.pquic_fec_parse_sfpid_frame.restype = C.c_uint32
    L.pquic_fec_write_recovered_frame.argtypes = [C.POINTER(C.c_uint64), C.c_uint8, C.c_void_p, C.c_void_p,
                                                  C.POINTER(C.c_size_t)]
    L.pquic_fec_parse_recovered_frame.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64),
                                                  C.POINTER(C.c_uint8)]
    L.pquic_fec_parse_recovered_frame.restype = C.c_void_p
    return L


def test_fec_frame_header_differential(lib, ref):
    rnd = random.Random(7001)
    for i in range(N):
        f = [rnd.randint(0, 1), rnd.choice([0, 1, 1200, 9000, 32767, rnd.randint(0, 32767)]), rnd.randint(0, 255),
             rnd.getrandbits(64), rnd.randint(0, 255), rnd.randint(0, 255)]
        rb = (C.c_uint8 * 32)()
        n = ref.ref_write_fec_frame_header(*f, rb)
        ob = (C.c_uint8 * 14)()
        assert lib.pquic_fec_write_fec_frame_header(C.byref(Hdr(*f)), ob) == n == 14, f
        assert bytes(ob) == bytes(rb[:n]), f
        raw = bytes([0x2A] + [rnd.getrandbits(8) for _ in range(13)])
        fields = (C.c_uint64 * 6)()
        ref.ref_parse_fec_frame_header((C.c_uint8 * 14).from_buffer_copy(raw), fields)
        h = Hdr()
        lib.pquic_fec_parse_fec_frame_header((C.c_uint8 * 14).from_buffer_copy(raw), C.byref(h))
        assert [h.fin, h.data_length, h.offset, h.repair_fpid_raw, h.nss, h.nrs] == list(fields), raw.hex()


def test_sfpid_frame_differential(lib, ref):
    rnd = random.Random(7002)
    for _ in range(N):
        raw, bmax = rnd.getrandbits(32), rnd.choice([0, 1, 4, 5, 8])
        rb = (C.c_uint8 * 8)()
        n = ref.ref_write_sfpid_frame(raw, rb, bmax)
        ob = (C.c_uint8 * 8)()
        got = C.c_size_t(0)
        ret = lib.pquic_fec_write_sfpid_frame(raw, ob, bmax, C.byref(got))
        if n < 0:  # the reference driver reports -error
            assert ret == -n, (raw, bmax)
        else:
            assert ret == 0 and got.value == n and bytes(ob[:n]) == bytes(rb[:n]), (raw, bmax)
        frame = bytes([0x29] + [rnd.getrandbits(8) for _ in range(4)])
        assert lib.pquic_fec_parse_sfpid_frame((C.c_uint8 * 5).from_buffer_copy(frame)) == \
            ref.ref_parse_sfpid_frame((C.c_uint8 * 5).from_buffer_copy(frame)), frame.hex()


def _packets(rnd):
    n = rnd.randint(0, 60)
    p = [rnd.getrandbits(rnd.choice([8, 40, 63, 64]))] if n else []
    for _ in range(n - 1):
        step = rnd.choice([1, 1, 2, 3, rnd.randint(1, 255), rnd.randint(256, 600), 0])
        p.append(min(p[-1] + step, 2**64 - 1))
    if p and rnd.random() < 0.05:  # not increasing: the writer must refuse as the reference does
        i = rnd.randrange(len(p))
        p[i] = rnd.getrandbits(64)
    return p


def test_recovered_frame_differential(lib, ref):
    rnd = random.Random(7003)
    written = []
    for _ in range(N):
        p = _packets(rnd)
        bmax = rnd.choice([0, 9, 10, 11, 64, 400, rnd.randint(0, 512)])
        pk = (C.c_uint64 * max(len(p), 1))(*p)
        rb = (C.c_uint8 * 512)()
        consumed = C.c_long(0)
        rret = ref.ref_write_recovered(pk, len(p), rb, bmax, C.byref(consumed))
        ob = (C.c_uint8 * 512)()
        got = C.c_size_t(0)
        base = C.addressof(ob)
        ret = lib.pquic_fec_write_recovered_frame(pk, len(p), base, base + bmax, C.byref(got))
        assert ret == rret and got.value == consumed.value, (p, bmax, ret, rret)
        assert bytes(ob[:got.value]) == bytes(rb[:consumed.value]), (p, bmax)
        if rret == 0 and consumed.value:
            written.append(bytes(rb[:consumed.value]))
    inputs = written[: N // 2]
    for _ in range(N // 2):  # crafted: type, count, LE u64 first, then range / gap bytes, sometimes cut short
        n = rnd.randint(0, 20)
        body = bytes([0x2B, n] + [rnd.getrandbits(8) for _ in range(8)] +
                     [rnd.choice([0, 1, 2, 3, 4, rnd.getrandbits(8)]) for _ in range(rnd.randint(0, 30))])
        if rnd.random() < 0.2:
            body = body[: rnd.randint(0, len(body))]
        inputs.append(body)
    for raw in inputs:
        buf = (C.c_uint8 * max(len(raw), 1)).from_buffer_copy(raw.ljust(max(len(raw), 1), b"\0"))
        rpk, opk = (C.c_uint64 * 256)(), (C.c_uint64 * 256)()
        rn, on = C.c_int(0), C.c_uint8(0)
        rend = ref.ref_parse_recovered(buf, len(raw), rpk, C.byref(rn))
        base = C.addressof(buf)
        oend = lib.pquic_fec_parse_recovered_frame(base, base + len(raw), opk, C.byref(on))
        if rend < 0:
            assert oend is None, raw.hex()
        else:
            assert oend is not None and oend - base == rend, raw.hex()
            assert list(opk[: on.value]) == list(rpk[: rn.value]), raw.hex()


def test_payload_to_source_symbol_differential(lib, ref):
    import gen_frames
    rnd = random.Random(7004)
    fn = lib.pquic_fec_payload_to_source_symbol
    fn.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64, C.c_void_p, SKIP_FN, C.c_void_p]
    fn.restype = C.c_uint32
    cb = SKIP_FN(synthetic_skip)
    for _ in range(N):
        pl = gen_frames.synthetic_payload(rnd)
        pn = rnd.getrandbits(64)
        src = (C.c_uint8 * max(len(pl), 1)).from_buffer_copy(pl.ljust(max(len(pl), 1), b"\0"))
        rb = (C.c_uint8 * (len(pl) + 16))()
        sl = C.c_uint32(0)
        rret = ref.ref_payload_to_source_symbol(src, len(pl), pn, rb, C.byref(sl))
        ob = (C.c_uint8 * (len(pl) + 16))()
        n = fn(C.addressof(src), len(pl), pn, C.addressof(ob), cb, None)
        assert n == rret and bytes(ob[:n]) == bytes(rb[:rret]), pl.hex()
