"""Generate tests/golden/cc_cases.json from the REFERENCE itself (survey container only).

Drives the reference pluglets protoops/maybe_notify_recovered_packets_to_cc.c
(fec_protoops.h:151-184) and protoops/process_simple_recovered_frame.c, compiled in place into
oracle/_ref/libfecref.so (`make -C oracle ref`), against scripted transports (ref_cc_scenario in
oracle/ref/ref_driver.c): every transport call the pluglet makes is logged.  The product's
pquic_fec_maybe_notify_recovered_packets_to_cc / pquic_fec_enqueue_recovered_packets must
reproduce the logs and the final ring state.

    python tests/golden/gen_cc.py
"""
from __future__ import annotations

import ctypes as C
import json
import os

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cc_cases.json")
NBUF = 50


def main():
    lib = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libfecref.so"))
    u64p, u32p, u8p = C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.POINTER(C.c_uint8)
    lib.ref_cc_scenario.argtypes = [C.c_int, u64p, u8p, u8p, C.c_uint64, C.c_uint64, C.c_uint64, u32p, u32p, u64p,
                                    u64p, C.c_int, u64p]
    lib.ref_process_recovered.argtypes = [u64p, C.c_int, u32p, u32p, u64p]
    rng = np.random.default_rng(2468)
    cases = []
    for t in range(300):
        n = int(rng.integers(0, 14))
        pns = np.cumsum(rng.integers(1, 4, n)).astype(np.uint64) + np.uint64(int(rng.integers(0, 1 << 40)))
        pure = (rng.random(n) < 0.2).astype(np.uint8)
        needed = (rng.random(n) < (0.9 if t % 4 else 0.5)).astype(np.uint8)
        # recovered numbers: some queued, some already gone (older / in gaps), some newer
        cand = list(pns) + [p - 1 for p in pns] + ([pns[-1] + 5] if n else [7])
        cand = sorted(set(int(x) for x in cand))
        m = int(rng.integers(0, min(len(cand), NBUF) + 1))
        rec = sorted(rng.choice(cand, m, replace=False).tolist()) if m else []
        if t % 7 == 3:
            rec = rec[::-1]  # out of order (the pluglet only ever peeks the oldest entry)
        start = int(rng.integers(0, NBUF))
        buf = np.zeros(NBUF, np.uint64)
        for i, p in enumerate(rec):
            buf[(start + i) % NBUF] = p
        srtt = int(rng.integers(1, 100000))
        latest = int(rng.integers(0, 1 << 30))
        now = latest + int(rng.integers(0, 2 * srtt)) if t % 5 else latest + srtt
        bs, bz = C.c_uint32(start), C.c_uint32(len(rec))
        bout = buf.copy()
        ev = np.zeros((256, 4), np.uint64)
        lat = C.c_uint64(0)
        nev = lib.ref_cc_scenario(n, pns.ctypes.data_as(u64p), pure.ctypes.data_as(u8p), needed.ctypes.data_as(u8p),
                                  srtt, latest, now, C.byref(bs), C.byref(bz), bout.ctypes.data_as(u64p),
                                  ev.ctypes.data_as(u64p), 256, C.byref(lat))
        assert nev <= 256
        cases.append({"pns": [int(x) for x in pns], "pure_ack": pure.tolist(), "needed": needed.tolist(),
                      "srtt": srtt, "latest": latest, "now": now, "buf_start": start,
                      "buf": [int(x) for x in buf], "buf_size": len(rec),
                      "events": ev[:nev].tolist(), "out_start": bs.value, "out_size": bz.value,
                      "out_buf": [int(x) for x in bout], "out_latest": lat.value})
    enq = []
    for t in range(60):  # the ring: RECOVERED frames of 0..40 packets into rings at every fill level
        start = int(rng.integers(0, NBUF))
        size = int(rng.integers(0, NBUF + 1))
        buf = rng.integers(0, 1 << 50, NBUF).astype(np.uint64)
        n = int(rng.integers(0, 41))
        pns = rng.integers(0, 1 << 50, n).astype(np.uint64)
        bs, bz = C.c_uint32(start), C.c_uint32(size)
        bout = buf.copy()
        lib.ref_process_recovered(pns.ctypes.data_as(u64p), n, C.byref(bs), C.byref(bz), bout.ctypes.data_as(u64p))
        enq.append({"start": start, "size": size, "buf": [int(x) for x in buf], "pns": [int(x) for x in pns],
                    "out_start": bs.value, "out_size": bz.value, "out_buf": [int(x) for x in bout]})
    with open(OUT, "w") as f:
        json.dump({"generated_by": "tests/golden/gen_cc.py (reference pluglets maybe_notify_recovered_packets_to_cc.c "
                                   "and process_simple_recovered_frame.c, native gcc, scripted transport)",
                   "event_kinds": {"1": "retransmit_needed_by_packet(pn, now, timer_based_in)",
                                   "2": "packet_was_lost(pn, path is the cnx path)",
                                   "3": "dequeue_retransmit_packet(pn, should_free)",
                                   "4": "congestion_algorithm_notify(notification, lost pn, now)",
                                   "5": "set latest CC notification time(t)"},
                   "notify": cases, "enqueue": enq}, f)
    kinds = {}
    for c in cases:
        for e in c["events"]:
            kinds[e[0]] = kinds.get(e[0], 0) + 1
    print(f"cc cases {len(cases)} (event kinds {kinds}), enqueue cases {len(enq)}")


if __name__ == "__main__":
    main()
