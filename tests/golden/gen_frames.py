"""Generate tests/golden/frames.json from the REFERENCE's frame code (survey container only).

Expected bytes come from the reference itself, built by `make -C oracle ref`:
  - FEC frame header: write_fec_frame_header / parse_fec_frame_header (plugins/fec/fec.h:175-194);
  - SFPID frame: helper_write_source_fpid_frame (fec_protoops.h:92-100) / parse_sfpid_frame (fec.h);
  - RECOVERED frame: the pluglets protoops/write_simple_recovered_frame.c and
    protoops/parse_simple_recovered_frame.c, run through get_cnx/set_cnx;
  - source symbols: the pluglet protoops/packet_payload_to_source_symbol.c, its skip_frame
    calls answered by the driver's synthetic frame grammar (ref_skip_frame_synthetic).
Inputs are seeded random values plus hand-made edge cases, stored verbatim.

    python tests/golden/gen_frames.py
"""
from __future__ import annotations

import ctypes as C
import json
import os
import random

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "frames.json")


def lib():
    L = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libfecref.so"))
    u8p, u64p = C.POINTER(C.c_uint8), C.POINTER(C.c_uint64)
    L.ref_write_fec_frame_header.argtypes = [C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int, C.c_int, u8p]
    L.ref_parse_fec_frame_header.argtypes = [u8p, u64p]
    L.ref_write_sfpid_frame.argtypes = [C.c_uint32, u8p, C.c_size_t]
    L.ref_parse_sfpid_frame.argtypes = [u8p]
    L.ref_parse_sfpid_frame.restype = C.c_uint32
    L.ref_write_recovered.argtypes = [u64p, C.c_int, u8p, C.c_long, C.POINTER(C.c_long)]
    L.ref_write_recovered.restype = C.c_long
    L.ref_parse_recovered.argtypes = [u8p, C.c_long, u64p, C.POINTER(C.c_int)]
    L.ref_parse_recovered.restype = C.c_long
    L.ref_payload_to_source_symbol.argtypes = [u8p, C.c_uint32, C.c_uint64, u8p, C.POINTER(C.c_uint32)]
    L.ref_payload_to_source_symbol.restype = C.c_long
    return L


def synthetic_payload(rnd):
    """A packet payload in the driver's synthetic frame grammar: PADDING runs, ACK (0x02),
    CRYPTO (0x06), STREAM-like (0x08-0x0f), SFPID (0x29), FEC (0x2a), others; sometimes a
    truncated last frame."""
    out = bytearray()
    for _ in range(rnd.randint(0, 12)):
        t = rnd.choice([0x00, 0x02, 0x06, 0x08, 0x0A, 0x0F, 0x29, 0x2A, 0x2B, 0x01, 0x1C, 0x30])
        if t == 0x00:
            out += bytes(rnd.randint(1, 20))
        else:
            n = rnd.choice([0, 1, 5, 20, 60, 200, rnd.randint(0, 255)])
            out += bytes([t, n]) + bytes(rnd.getrandbits(8) for _ in range(n))
    if rnd.random() < 0.2 and len(out) > 3:
        out = out[: rnd.randint(1, len(out))]
    return bytes(out)


def main():
    L = lib()
    rnd = random.Random(20261015)
    out = {"fec_header_write": [], "fec_header_parse": [], "sfpid_write": [], "sfpid_parse": [],
           "recovered_write": [], "recovered_parse": []}
    for i in range(200):
        f = [rnd.randint(0, 1), rnd.choice([0, 1, 1200, 1400, 9000, 32767, rnd.randint(0, 32767)]),
             rnd.randint(0, 255), rnd.getrandbits(64), rnd.randint(0, 255), rnd.randint(0, 255)]
        if i < 3:
            f = [[1, 1200, 1, 0xDEADBEEF12345603, 16, 4], [0, 0, 0, 0, 0, 0], [1, 32767, 255, 2**64 - 1, 255, 255]][i]
        buf = (C.c_uint8 * 32)()
        n = L.ref_write_fec_frame_header(*f, buf)
        out["fec_header_write"].append({"fields": f, "bytes": bytes(buf[:n]).hex()})
    for i in range(100):
        raw = bytes([0x2A] + [rnd.getrandbits(8) for _ in range(13)])
        fields = (C.c_uint64 * 6)()
        L.ref_parse_fec_frame_header((C.c_uint8 * 14).from_buffer_copy(raw), fields)
        out["fec_header_parse"].append({"bytes": raw.hex(), "fields": list(fields)})
    for i in range(50):
        raw = rnd.getrandbits(32) if i else 0x12345603
        buf = (C.c_uint8 * 8)()
        bmax = rnd.choice([5, 8, 4, 0]) if i > 3 else 5
        n = L.ref_write_sfpid_frame(raw, buf, bmax)
        out["sfpid_write"].append({"raw": raw, "bytes_max": bmax, "ret": n, "bytes": bytes(buf[:max(n, 0)]).hex()})
    for i in range(50):
        raw = bytes([0x29] + [rnd.getrandbits(8) for _ in range(4)])
        v = L.ref_parse_sfpid_frame((C.c_uint8 * 5).from_buffer_copy(raw))
        out["sfpid_parse"].append({"bytes": raw.hex(), "raw": v})
    # RECOVERED frames: edge cases then random increasing lists (gaps 1..255), some invalid
    cases = [[], [5], [5, 6], [5, 7, 8, 300], [10, 10], [10, 9], [100, 356], [100, 355], [2**63, 2**63 + 1]]
    for _ in range(60):
        n = rnd.randint(1, 40)
        p = [rnd.getrandbits(40)]
        for _ in range(n - 1):
            p.append(p[-1] + rnd.choice([1, 1, 2, 3, rnd.randint(1, 255)]))
        cases.append(p)
    for p in cases:
        for bmax in (64, 400, 10, 9):
            pk = (C.c_uint64 * max(len(p), 1))(*p)
            buf = (C.c_uint8 * 512)()
            consumed = C.c_long(0)
            ret = L.ref_write_recovered(pk, len(p), buf, bmax, C.byref(consumed))
            out["recovered_write"].append({"packets": p, "bytes_max": bmax, "ret": ret, "consumed": consumed.value,
                                           "bytes": bytes(buf[:consumed.value]).hex()})
    parse_inputs = [w["bytes"] for w in out["recovered_write"] if w["ret"] == 0][:80]
    for _ in range(60):  # crafted: type, n, LE u64 first, then ranges/gaps
        n = rnd.randint(1, 12)
        body = [0x2B, n] + [rnd.getrandbits(8) for _ in range(8)] + [rnd.randint(0, 4) for _ in range(rnd.randint(0, 14))]
        parse_inputs.append(bytes(body).hex())
    parse_inputs += ["2b01" + "00" * 8, "2b02" + "11" * 8, "2b", "2b0300" + "ff" * 7 + "0102"]
    for h in parse_inputs:
        raw = bytes.fromhex(h)
        pk = (C.c_uint64 * 256)()
        n = C.c_int(0)
        src = (C.c_uint8 * max(len(raw), 1)).from_buffer_copy(raw.ljust(max(len(raw), 1), b"\0"))
        end = L.ref_parse_recovered(src, len(raw), pk, C.byref(n))
        out["recovered_parse"].append({"bytes": h, "consumed": end, "packets": list(pk[: n.value])})
    rs = random.Random(20261016)  # separate stream: the sections above stay byte-identical
    out["source_symbol"] = []
    payloads = [b"", bytes([0x02, 0x03, 1, 2, 3]), bytes(16), bytes([0x08, 2, 7, 7, 0, 0, 0x06, 1, 9])]
    payloads += [synthetic_payload(rs) for _ in range(120)]
    for i, pl in enumerate(payloads):
        pn = rs.getrandbits(64) if i else 0x0102030405060708
        src = (C.c_uint8 * max(len(pl), 1)).from_buffer_copy(pl.ljust(max(len(pl), 1), b"\0"))
        buf = (C.c_uint8 * (len(pl) + 16))()
        sl = C.c_uint32(0)
        ret = L.ref_payload_to_source_symbol(src, len(pl), pn, buf, C.byref(sl))
        out["source_symbol"].append({"payload": pl.hex(), "pn": pn, "ret": ret, "symbol": bytes(buf[:ret]).hex(),
                                     "state_current_symbol_length": sl.value})
    with open(OUT, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", OUT, {k: len(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
