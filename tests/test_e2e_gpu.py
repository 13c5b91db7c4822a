"""End to end over the whole FEC path, sender to receiver, through the engine's batching adapter on
the GPU:

  packets (synthetic frame grammar) -> source symbols through the packet_payload_to_source_symbol
  protoop -> blocks of k symbols -> batched fec_generate_repair_symbols -> FEC frames (one per
  repair symbol, as block_framework_sender.h:100 sends them: piece offset 1, fin set) -> a lossy
  channel -> parsed FEC frames -> batched fec_recover -> recovered symbols -> packet numbers from
  the symbol prefix -> a RECOVERED frame, written and parsed back.

Every recovered symbol is checked against the oracle's decode of the same received set and against
the sender's own symbol (zero-padded to the block's repair length); the packet numbers must round
trip through the RECOVERED frame.  Blocks mix RLC k=16 r=4, RLC k=8 r=2 and XOR k=4 r=1."""
import ctypes as C
import os

import numpy as np
import pytest

from oracle_py import DEC_RECOVERED, Oracle
from test_batch_gpu import Batch
from test_frames import Hdr

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
LIB = os.path.join(ROOT, "pquic_amd", "lib", "libpquic_fec.so")

# frame types the capture keeps (anything but 0x00 PADDING, 0x02 ACK, 0x06 CRYPTO_HS)
KEPT_TYPES = [0x01, 0x04, 0x05, 0x08, 0x0a, 0x0d, 0x0f, 0x10, 0x1c]


def _frames_lib():
    L = C.CDLL(LIB)
    u8p = C.POINTER(C.c_uint8)
    L.pquic_fec_write_fec_frame_header.argtypes = [C.POINTER(Hdr), u8p]
    L.pquic_fec_write_fec_frame_header.restype = C.c_size_t
    L.pquic_fec_parse_fec_frame_header.argtypes = [u8p, C.POINTER(Hdr)]
    L.pquic_fec_write_recovered_frame.argtypes = [C.POINTER(C.c_uint64), C.c_uint8, C.c_void_p, C.c_void_p,
                                                  C.POINTER(C.c_size_t)]
    L.pquic_fec_parse_recovered_frame.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64),
                                                  C.POINTER(C.c_uint8)]
    L.pquic_fec_parse_recovered_frame.restype = C.c_void_p
    return L


def _payload(rng, target):
    """One packet payload: a few kept frames, sometimes an ACK or CRYPTO frame (dropped by the
    capture) and trailing PADDING."""
    out = bytearray()
    while len(out) < target:
        t = int(rng.choice(KEPT_TYPES)) if rng.random() > 0.2 else int(rng.choice([0x02, 0x06]))
        n = int(rng.integers(0, min(255, max(1, target - len(out))) + 1))
        out += bytes([t, n]) + rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    if rng.random() < 0.3:
        out += bytes(int(rng.integers(1, 40)))
    return bytes(out)


def _capture(mh, payload, pn):
    src = (C.c_uint8 * max(len(payload), 1)).from_buffer_copy(payload.ljust(max(len(payload), 1), b"\0"))
    buf = (C.c_uint8 * (len(payload) + 16))()
    n = mh.mh_payload_to_source_symbol(C.addressof(src), len(payload), pn, C.addressof(buf))
    assert 9 <= n <= len(payload) + 9
    sym = bytes(buf[:n])
    assert sym[0] == 0x10 and int.from_bytes(sym[1:9], "big") == pn
    return np.frombuffer(sym, np.uint8).copy()


def _fec_frames(fl, reps, fpids, k, r):
    frames = []
    for rep, fpid in zip(reps, fpids):
        h = Hdr(1, len(rep), 1, fpid, k, r)
        hb = (C.c_uint8 * 14)()
        assert fl.pquic_fec_write_fec_frame_header(C.byref(h), hb) == 14
        frames.append(bytes(hb) + rep.tobytes())
    return frames


def _parse_fec_frame(fl, frame):
    h = Hdr()
    fl.pquic_fec_parse_fec_frame_header((C.c_uint8 * 14).from_buffer_copy(frame[:14]), C.byref(h))
    assert frame[0] == 0x2a and h.fin == 1 and h.offset == 1
    return h, np.frombuffer(frame[14:14 + h.data_length], np.uint8).copy()


@pytest.mark.parametrize("seed,loss", [(1, 0.08), (2, 0.2), (3, 0.35)])
def test_sender_channel_receiver(seed, loss):
    rng = np.random.default_rng(seed)
    o = Oracle()
    fl = _frames_lib()
    tx = Batch(8, max_delay_us=200)
    mh = tx.L
    mh.mh_payload_to_source_symbol.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64, C.c_void_p]
    mh.mh_payload_to_source_symbol.restype = C.c_long

    # --- sender: packets -> source symbols -> blocks -> repair symbols -> FEC frames
    blocks = []
    pn = 1000 * seed
    for b in range(36):
        xor, k, r = [(False, 16, 4), (False, 8, 2), (True, 4, 1)][b % 3]
        fbn = (seed << 16) | b
        pns = list(range(pn, pn + k))
        pn += k
        size = int(rng.choice([60, 400, 1200, 1350]))
        syms = [_capture(mh, _payload(rng, int(rng.integers(size // 2, size + 1))), p) for p in pns]
        blocks.append(dict(xor=xor, k=k, r=r, fbn=fbn, pns=pns, syms=syms,
                           ticket=tx.generate(xor, fbn, syms, r, now=b)))
    mh.mh_batch_drain()
    for blk in blocks:
        assert tx.status(blk["ticket"]) == (0, 1)
        reps, fpids = tx.repairs(blk["ticket"])
        assert fpids == [(blk["fbn"] << 8) | i for i in range(blk["r"])]
        L = max(len(s) for s in blk["syms"])
        pad = [np.pad(s, (0, L - len(s))) for s in blk["syms"]]
        want = [o.xor_encode_block(pad)[1]] if blk["xor"] else o.rlc_encode_block(blk["fbn"], pad, blk["r"])[1]
        assert [x.tobytes() for x in reps] == [x.tobytes() for x in want]
        blk["frames"] = _fec_frames(fl, reps, fpids, blk["k"], blk["r"])
    tx.close()

    # --- channel: independent losses on source packets and FEC frames
    rx = Batch(16, max_delay_us=200)
    recovered_pns = []
    n_rec = 0
    for i, blk in enumerate(blocks):
        k, r, fbn = blk["k"], blk["r"], blk["fbn"]
        srcs = [None if rng.random() < loss else s for s in blk["syms"]]
        reps, fpids = [None] * r, [0] * r
        for fr in blk["frames"]:
            if rng.random() < loss:
                continue
            h, data = _parse_fec_frame(fl, fr)  # --- receiver side from here
            assert (h.nss, h.nrs) == (k, r) and h.repair_fpid_raw >> 8 == fbn
            idx = h.repair_fpid_raw & 0xFF
            reps[idx], fpids[idx] = data, h.repair_fpid_raw
        blk["rx"] = (srcs, reps)
        blk["rx_ticket"] = rx.recover(blk["xor"], fbn, srcs, reps, [f or ((fbn << 8) | j) for j, f in
                                                                      enumerate(fpids)], now=i)
    rx.L.mh_batch_drain()
    for blk in blocks:
        k, srcs, reps = blk["k"], *blk["rx"]
        ret, calls = rx.status(blk["rx_ticket"])
        assert calls == 1
        rec, cur = rx.recovered(blk["rx_ticket"])
        if blk["xor"]:
            st, want = o.xor_decode_block(srcs, reps)
        else:
            st, want = o.rlc_decode_block(blk["fbn"], srcs, reps)
            assert ret == 0
            assert cur == sum(s is not None for s in srcs) + len(rec)
        if st != DEC_RECOVERED:
            want = {}
        assert sorted(rec) == sorted(want), blk["fbn"]
        for j, sym in rec.items():
            assert srcs[j] is None
            assert sym.tobytes() == want[j].tobytes()
            orig = blk["syms"][j]
            assert sym[: len(orig)].tobytes() == orig.tobytes() and not sym[len(orig):].any()
            recovered_pns.append(int.from_bytes(sym[1:9].tobytes(), "big"))
            assert recovered_pns[-1] == blk["pns"][j]
            n_rec += 1
    st = rx.stats()
    assert st["engine_errors"] == 0
    rx.close()
    assert n_rec > 0

    # --- RECOVERED frames carrying the recovered packet numbers, in 40-number chunks
    # (a new frame whenever the gap exceeds 255, which the writer refuses: :47)
    pns = sorted(recovered_pns)
    chunks = [[pns[0]]]
    for a, b in zip(pns, pns[1:]):
        if b - a > 0xFF or len(chunks[-1]) == 40:
            chunks.append([])
        chunks[-1].append(b)
    for chunk in chunks:
        pk = (C.c_uint64 * len(chunk))(*chunk)
        buf = (C.c_uint8 * 1024)()
        n = C.c_size_t(0)
        base = C.addressof(buf)
        assert fl.pquic_fec_write_recovered_frame(pk, len(chunk), base, base + 1024, C.byref(n)) == 0
        out = (C.c_uint64 * 256)()
        cnt = C.c_uint8(0)
        end = fl.pquic_fec_parse_recovered_frame(base, base + n.value, out, C.byref(cnt))
        assert end is not None and end - base == n.value and cnt.value == len(chunk)
        # The reference's writer and parser disagree on the gap byte: the writer stores the
        # difference d (write_simple_recovered_frame.c:68), the parser skips (d + 1) mod 256 and
        # then one more (parse_simple_recovered_frame.c:66-68).  The receiver sees that numbering.
        want = [chunk[0]]
        for a, b in zip(chunk, chunk[1:]):
            want.append(want[-1] + ((b - a + 1) & 0xFF) + 1)
        assert list(out[: cnt.value]) == want
