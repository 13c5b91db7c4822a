"""Recovered packets -> congestion control (include/pquic_fec_cc.h), CPU only.

The product's pquic_fec_maybe_notify_recovered_packets_to_cc and pquic_fec_enqueue_recovered_packets,
bound to a scripted transport (tests/host/mini_host.c), must make exactly the transport calls the
reference pluglets make (protoops/maybe_notify_recovered_packets_to_cc.c, fec_protoops.h:151-184;
protoops/process_simple_recovered_frame.c) and leave the same ring: tests/golden/cc_cases.json,
produced by those pluglets compiled natively (tests/golden/gen_cc.py)."""
import ctypes as C
import os

import numpy as np
import pytest

from golden_io import load

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
# PQUIC_TEST_MINIHOST: a sanitizer build over the CPU engine stand-in (tests/sanitize, test_sanitize.py)
MINIHOST = os.environ.get("PQUIC_TEST_MINIHOST") or os.path.join(ROOT, "tests", "host", "libminihost.so")
u64p, u32p, u8p = C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.POINTER(C.c_uint8)


@pytest.fixture(scope="module")
def mh():
    lib = C.CDLL(MINIHOST)
    lib.mh_cc_scenario.argtypes = [C.c_int, u64p, u8p, u8p, C.c_uint64, C.c_uint64, C.c_uint64, u32p, u32p, u64p,
                                   u64p, C.c_int, u64p]
    lib.mh_process_recovered.argtypes = [u64p, C.c_int, u32p, u32p, u64p]
    return lib


def test_notify_matches_reference_event_logs(mh):
    d = load("cc_cases.json")
    kinds = set()
    for i, c in enumerate(d["notify"]):
        pns = np.array(c["pns"], np.uint64)
        pure = np.array(c["pure_ack"], np.uint8)
        needed = np.array(c["needed"], np.uint8)
        buf = np.array(c["buf"], np.uint64)
        bs, bz = C.c_uint32(c["buf_start"]), C.c_uint32(c["buf_size"])
        ev = np.zeros((256, 4), np.uint64)
        lat = C.c_uint64(0)
        nev = mh.mh_cc_scenario(len(pns), pns.ctypes.data_as(u64p), pure.ctypes.data_as(u8p),
                                needed.ctypes.data_as(u8p), c["srtt"], c["latest"], c["now"], C.byref(bs),
                                C.byref(bz), buf.ctypes.data_as(u64p), ev.ctypes.data_as(u64p), 256, C.byref(lat))
        assert ev[:nev].tolist() == c["events"], i
        assert (bs.value, bz.value, lat.value) == (c["out_start"], c["out_size"], c["out_latest"]), i
        assert [int(x) for x in buf] == c["out_buf"], i
        kinds |= {e[0] for e in c["events"]}
    assert kinds == {1, 2, 3, 4, 5}  # every transport call kind is exercised


def test_enqueue_ring_matches_reference(mh):
    d = load("cc_cases.json")
    wrapped = 0
    for i, c in enumerate(d["enqueue"]):
        buf = np.array(c["buf"], np.uint64)
        pns = np.array(c["pns"], np.uint64)
        bs, bz = C.c_uint32(c["start"]), C.c_uint32(c["size"])
        mh.mh_process_recovered(pns.ctypes.data_as(u64p), len(pns), C.byref(bs), C.byref(bz),
                                buf.ctypes.data_as(u64p))
        assert (bs.value, bz.value) == (c["out_start"], c["out_size"]), i
        assert [int(x) for x in buf] == c["out_buf"], i
        wrapped += c["size"] + len(c["pns"]) > 50
    assert wrapped > 5  # full rings drop their oldest entries
