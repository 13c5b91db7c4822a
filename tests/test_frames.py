"""Frame codecs (include/pquic_fec_frames.h) against golden vectors produced by the reference's
own frame code (tests/golden/gen_frames.py): FEC frame header, SOURCE_FPID frame, RECOVERED
frame (quirks included) and the source-symbol prefix.  Pure host C: runs without a GPU."""
import ctypes as C
import json
import os

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
# PQUIC_TEST_MINIHOST: the frame codecs from a sanitizer build (tests/sanitize, test_sanitize.py)
LIB = os.environ.get("PQUIC_TEST_MINIHOST") or os.path.join(ROOT, "pquic_amd", "lib", "libpquic_fec.so")
GOLD = os.path.join(ROOT, "tests", "golden", "frames.json")


class Hdr(C.Structure):
    _fields_ = [("fin", C.c_uint8), ("data_length", C.c_uint16), ("offset", C.c_uint8),
                ("repair_fpid_raw", C.c_uint64), ("nss", C.c_uint8), ("nrs", C.c_uint8)]


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.skip("engine library not built")
    L = C.CDLL(LIB)
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
    L.pquic_fec_source_symbol_header.argtypes = [C.c_uint64, u8p]
    return L


@pytest.fixture(scope="module")
def gold():
    with open(GOLD) as f:
        return json.load(f)


def test_fec_frame_header(lib, gold):
    for case in gold["fec_header_write"]:
        fin, ln, off, raw, nss, nrs = case["fields"]
        h = Hdr(fin, ln, off, raw, nss, nrs)
        buf = (C.c_uint8 * 14)()
        assert lib.pquic_fec_write_fec_frame_header(C.byref(h), buf) == 14
        assert bytes(buf).hex() == case["bytes"]
    for case in gold["fec_header_parse"]:
        raw = bytes.fromhex(case["bytes"])
        h = Hdr()
        lib.pquic_fec_parse_fec_frame_header((C.c_uint8 * 14).from_buffer_copy(raw), C.byref(h))
        assert [h.fin, h.data_length, h.offset, h.repair_fpid_raw, h.nss, h.nrs] == case["fields"]
    # fin=1 len=1200 -> 0x0961; repair FPID raw packing 0xdeadbeef12345603
    assert gold["fec_header_write"][0]["bytes"].startswith("2a0961")


def test_sfpid_frame(lib, gold):
    for case in gold["sfpid_write"]:
        buf = (C.c_uint8 * 8)()
        n = C.c_size_t(0)
        ret = lib.pquic_fec_write_sfpid_frame(case["raw"], buf, case["bytes_max"], C.byref(n))
        if case["ret"] < 0:  # the reference driver reports -error
            assert ret == -case["ret"]
        else:
            assert ret == 0 and n.value == case["ret"] and bytes(buf[: n.value]).hex() == case["bytes"]
    for case in gold["sfpid_parse"]:
        raw = bytes.fromhex(case["bytes"])
        assert lib.pquic_fec_parse_sfpid_frame((C.c_uint8 * 5).from_buffer_copy(raw)) == case["raw"]


def test_recovered_frame_write(lib, gold):
    for case in gold["recovered_write"]:
        p = case["packets"]
        pk = (C.c_uint64 * max(len(p), 1))(*p)
        buf = (C.c_uint8 * 512)()
        n = C.c_size_t(0)
        base = C.addressof(buf)
        ret = lib.pquic_fec_write_recovered_frame(pk, len(p), base, base + case["bytes_max"], C.byref(n))
        assert ret == case["ret"], case
        assert n.value == case["consumed"]
        assert bytes(buf[: n.value]).hex() == case["bytes"]


def test_recovered_frame_parse(lib, gold):
    for case in gold["recovered_parse"]:
        raw = bytes.fromhex(case["bytes"])
        buf = (C.c_uint8 * max(len(raw), 1)).from_buffer_copy(raw.ljust(max(len(raw), 1), b"\0"))
        pk = (C.c_uint64 * 256)()
        n = C.c_uint8(0)
        base = C.addressof(buf)
        end = lib.pquic_fec_parse_recovered_frame(base, base + len(raw), pk, C.byref(n))
        if case["consumed"] < 0:
            assert end is None, case
        else:
            assert end - base == case["consumed"], case
            assert list(pk[: n.value]) == case["packets"], case


def test_source_symbol_header(lib):
    buf = (C.c_uint8 * 9)()
    assert lib.pquic_fec_source_symbol_header(0x0102030405060708, buf) == 9
    assert bytes(buf).hex() == "10" + "0102030405060708"


SKIP_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint8), C.c_size_t, C.POINTER(C.c_size_t),
                      C.POINTER(C.c_int))


def synthetic_skip(ctx, bytes_, bytes_max, consumed, pure_ack):
    """The frame grammar the reference pluglet was driven with (oracle/ref/ref_driver.c
    ref_skip_frame_synthetic): PADDING runs of 0x00, every other type [type][len][len bytes]."""
    pure_ack[0] = 0
    if bytes_max == 0:
        consumed[0] = 0
        return -1
    if bytes_[0] == 0:
        n = 1
        while n < bytes_max and bytes_[n] == 0:
            n += 1
    else:
        n = bytes_max if bytes_max < 2 else min(bytes_max, 2 + bytes_[1])
    consumed[0] = n
    return 0


def test_payload_to_source_symbol(lib, gold):
    """packet_payload_to_source_symbol.c: symbol bytes and length equal the reference pluglet's
    on 124 payloads (ACK / PADDING / CRYPTO frames dropped, truncated last frames, empty)."""
    fn = lib.pquic_fec_payload_to_source_symbol
    fn.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64, C.c_void_p, SKIP_FN, C.c_void_p]
    fn.restype = C.c_uint32
    cb = SKIP_FN(synthetic_skip)
    for case in gold["source_symbol"]:
        pl = bytes.fromhex(case["payload"])
        src = (C.c_uint8 * max(len(pl), 1)).from_buffer_copy(pl.ljust(max(len(pl), 1), b"\0"))
        buf = (C.c_uint8 * (len(pl) + 16))()
        n = fn(C.addressof(src), len(pl), case["pn"], C.addressof(buf), cb, None)
        assert n == case["ret"], case
        assert bytes(buf[:n]).hex() == case["symbol"], case
    assert any(len(c["symbol"]) // 2 < 9 + len(c["payload"]) // 2 for c in gold["source_symbol"])


def test_payload_to_source_symbol_protoop():
    """The protoop adapter (inputs through get_cnx, frames through the host's skip_frame) on the
    same vectors, driven by the picoquic stand-in; a NULL buffer returns PICOQUIC_ERROR_MEMORY."""
    so = os.environ.get("PQUIC_TEST_MINIHOST") or os.path.join(ROOT, "tests", "host", "libminihost.so")
    if not os.path.exists(so):
        pytest.skip("mini host not built")
    M = C.CDLL(so)
    M.mh_payload_to_source_symbol.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64, C.c_void_p]
    M.mh_payload_to_source_symbol.restype = C.c_long
    M.mh_unbind()
    assert M.mh_payload_to_source_symbol(None, 0, 0, None) == 0x41B  # unbound
    assert M.mh_bind(0) == 0
    with open(GOLD) as f:
        cases = json.load(f)["source_symbol"]
    for case in cases:
        pl = bytes.fromhex(case["payload"])
        src = (C.c_uint8 * max(len(pl), 1)).from_buffer_copy(pl.ljust(max(len(pl), 1), b"\0"))
        buf = (C.c_uint8 * (len(pl) + 16))()
        n = M.mh_payload_to_source_symbol(C.addressof(src), len(pl), case["pn"], C.addressof(buf))
        assert n == case["ret"] and bytes(buf[:n]).hex() == case["symbol"], case
    assert M.mh_payload_to_source_symbol(C.addressof(src), 4, 1, None) == 0x405
    M.mh_unbind()


@pytest.mark.gpu
@pytest.mark.parametrize("nb,r,L,dlen,stride", [(257, 4, 1200, 1200, 1216), (33, 8, 1200, 1000, 1400),
                                                (5, 16, 9000, 8998, 9016), (64, 1, 8, 3, 20),
                                                (33, 8, 1200, 1000, 1216), (40, 3, 1600, 1590, 1616)])
def test_device_repair_frames(lib, nb, r, L, dlen, stride):
    """fecgpu_write_repair_frames vs the host codec (itself pinned to the reference) + payload."""
    import numpy as np
    import torch
    from pquic_amd import Engine
    eng = Engine(0)
    rng = np.random.default_rng(nb)
    rep_h = rng.integers(0, 256, (nb, r, L), dtype=np.uint8)
    fbn = rng.integers(0, 1 << 24, nb, dtype=np.uint32)
    frames = torch.full((nb * r * stride,), 0xCC, dtype=torch.uint8, device="cuda:0")
    eng.write_repair_frames(torch.from_numpy(rep_h).cuda(), frames, nb, r, L, dlen, stride, 16, r,
                            fbn=torch.from_numpy(fbn.view(np.int32)).cuda())
    got = frames.cpu().numpy().reshape(nb * r, stride)
    for b in range(nb):
        for i in range(r):
            h = Hdr(1, dlen, 1, (int(fbn[b]) << 8) | i, 16, r)
            buf = (C.c_uint8 * 14)()
            lib.pquic_fec_write_fec_frame_header(C.byref(h), buf)
            f = got[b * r + i]
            assert bytes(f[:14]) == bytes(buf), (b, i)
            assert np.array_equal(f[14:14 + dlen], rep_h[b, i, :dlen]), (b, i)
            assert not f[14 + dlen:].any(), (b, i)
