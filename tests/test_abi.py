"""C-ABI boundary checks that need no GPU: the engine library loads, exports every entry
point declared in include/*.h, validates arguments without touching a device, matches the
reference's fec_block_t layout, and refuses to compute when no gfx950 device is present
(there is no CPU fallback in the product path)."""
import ctypes as C
import os
import re

import pytest

from golden_io import load

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
LIB = os.path.join(ROOT, "pquic_amd", "lib", "libpquic_fec.so")
# PQUIC_TEST_MINIHOST: a sanitizer build over the CPU engine stand-in (tests/sanitize, test_sanitize.py)
MINIHOST = os.environ.get("PQUIC_TEST_MINIHOST") or os.path.join(ROOT, "tests", "host", "libminihost.so")


def declared_functions():
    names = set()
    for h in sorted(f for f in os.listdir(os.path.join(ROOT, "include")) if f.endswith(".h")):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b((?:fecgpu|pquic_fec)_\w+)\s*\(", text, re.M):
            if not m.group(0).lstrip().startswith("typedef"):
                names.add(m.group(1))
    return sorted(names)


@pytest.fixture(scope="module")
def lib():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"
    return C.CDLL(LIB)


def test_exports_every_declared_symbol(lib):
    names = declared_functions()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_layout_matches_reference(lib):
    lay = load("layout.json")
    out = (C.c_uint64 * 8)()
    assert lib.pquic_fec_layout(out) == 8
    exp = [lay["sizeof_fec_block_t"], lay["sizeof_source_symbol_t"], lay["sizeof_repair_symbol_t"],
           lay["off_source_symbols"], lay["off_repair_symbols"], lay["off_source_data"],
           lay["off_repair_data"], lay["sizeof_repair_fpid_t"]]
    assert list(out) == exp


def test_argument_validation_without_device(lib):
    lib.fecgpu_rlc_encode.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32,
                                      C.c_uint32, C.c_void_p, C.c_void_p]
    assert lib.fecgpu_rlc_encode(None, None, 0, 4, 1, 1200, 0, None, None) == 0      # empty batch
    assert lib.fecgpu_rlc_encode(None, None, 1, 4, 1, 1200, 0, None, None) == -1     # NULL buffers
    assert lib.fecgpu_rlc_encode(16, 16, 1, 4, 1, 1201, 0, None, None) == -1         # L % 4
    assert lib.fecgpu_rlc_encode(16, 16, 1, 0, 1, 1200, 0, None, None) == -1         # k = 0
    assert lib.fecgpu_rlc_encode(16, 16, 1, 129, 1, 1200, 0, None, None) == -1       # k > 128
    lib.fecgpu_rlc_decode_workspace.restype = C.c_size_t
    lib.fecgpu_rlc_decode_workspace.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32]
    assert lib.fecgpu_rlc_decode_workspace(1000, 16, 4) >= 1000 * (16 * 4 + 16)
    lib.fecgpu_version.restype = C.c_char_p
    assert b"gfx950" in lib.fecgpu_version()


def test_no_cpu_fallback(lib):
    """Without a gfx950 device the engine reports NO_DEVICE and the protoop adapters fail
    with an error code instead of computing on the CPU."""
    if lib.fecgpu_init(0) == 0:
        pytest.skip("a gfx950 device is present here")
    assert lib.fecgpu_init(0) == -3
    mh = C.CDLL(MINIHOST)
    mh.mh_generate.restype = C.c_long
    import numpy as np
    k, r, L = 4, 2, 64
    src = np.arange(k * L, dtype=np.uint8)
    lens = np.full(k, L, np.uint16)
    rep = np.zeros(r * L, np.uint8)
    rl = np.zeros(r, np.uint16)
    fp = np.zeros(r, np.uint64)
    sch = np.zeros(2, np.uint64)
    p = lambda a, t=C.c_uint8: a.ctypes.data_as(C.POINTER(t))  # noqa: E731
    # unbound: the documented error code
    mh.mh_unbind()
    assert mh.mh_generate(0, 7, k, r, p(src), p(lens, C.c_uint16), L, p(rep), p(rl, C.c_uint16),
                          p(fp, C.c_uint64), L, p(sch, C.c_uint64)) == 0x41B
    mh.mh_bind(0)
    before = mh.mh_live_allocations()
    ret = mh.mh_generate(0, 7, k, r, p(src), p(lens, C.c_uint16), L, p(rep), p(rl, C.c_uint16),
                         p(fp, C.c_uint64), L, p(sch, C.c_uint64))
    assert ret == 0x41B and not rep.any()
    assert mh.mh_live_allocations() == before


def test_integration_stub_compiles_against_picoquic(tmp_path):
    """INTEGRATION.md's binding (both options) compiles against picoquic's own headers
    (survey container only; the reference tree is not on the GPU box)."""
    import subprocess
    pico = "/root/reference/picoquic"
    if not os.path.isdir(pico):
        pytest.skip("reference tree not present")
    r = subprocess.run(["gcc", "-std=gnu11", "-c", "-Wall", "-Werror", f"-I{pico}",
                        f"-I{os.path.join(ROOT, 'include')}", os.path.join(ROOT, "tests", "host", "integration_stub.c"),
                        "-o", str(tmp_path / "stub.o")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_integration_option_b_allocates_in_the_inserted_fec_plugin(tmp_path):
    """INTEGRATION.md §4 (Option B): the native create_fec_schemes registered by the stub allocates its
    scheme in the arena of the FEC composition the host inserted -- under each shipped manifest name
    (fec.plugin:1, fec_rlc_gf256_window.plugin:1, fec_rlc_gf256_window_protect_end_of_stream_only_
    inflight.plugin:1), given at install or found by prefix -- and never in another plugin's; a
    connection without a FEC plugin gets PICOQUIC_ERROR_MEMORY, not a NULL dereference.  Built against
    picoquic's own headers and structures (survey container only), run on the CPU (no device call)."""
    import subprocess
    pico = "/root/reference/picoquic"
    if not os.path.isdir(pico):
        pytest.skip("reference tree not present")
    exe = str(tmp_path / "integration_driver")
    lib = os.path.join(ROOT, "pquic_amd", "lib")
    r = subprocess.run(["gcc", "-std=gnu11", "-Wall", "-Werror", f"-I{pico}", f"-I{os.path.join(ROOT, 'include')}",
                        os.path.join(ROOT, "tests", "host", "integration_driver.c"), f"-L{lib}", "-lpquic_fec",
                        f"-Wl,-rpath,{lib}", "-o", exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(" ok\n") == 8 and "all ok" in r.stdout


def test_oversized_block_rejected_without_device_call():
    """Totals above the block's 100 symbol slots (nss / nrs come from the peer,
    block_framework_receiver.h:44-45) are refused before any engine call -- the reference reads
    past fec_block_t there.  Runs on any host: a refused block never reaches the device, so the
    operation counters do not move while the error counter does."""
    import numpy as np
    mh = C.CDLL(MINIHOST)
    mh.mh_oversized.restype = C.c_long
    assert mh.mh_bind(0) == 0
    st0 = np.zeros(5, np.uint64)
    mh.mh_protoop_stats(st0.ctypes.data_as(C.POINTER(C.c_uint64)))
    for xor, op, kt, rt in [(0, 0, 150, 4), (0, 0, 16, 120), (0, 1, 150, 20), (0, 1, 100, 101), (1, 1, 150, 1),
                            (1, 0, 150, 1)]:
        assert mh.mh_oversized(xor, op, kt, rt) == 0x41B
    st1 = np.zeros(5, np.uint64)
    mh.mh_protoop_stats(st1.ctypes.data_as(C.POINTER(C.c_uint64)))
    assert st1[0] == st0[0] and st1[1] == st0[1]
    assert st1[4] == st0[4] + 6


def test_generated_bodies_match_generator(tmp_path):
    """pquic_amd/csrc/bitslice_gen.h is exactly what gen_bitslice.py writes with its defaults (the
    generator also self-checks the plane algebra and the transpose against a byte-level GF model)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    gen = os.path.join(root, "pquic_amd", "csrc", "gen_bitslice.py")
    out = tmp_path / "bitslice_gen.h"
    env = {k: v for k, v in os.environ.items() if not k.startswith("FEC_GEN")}
    env["FEC_GEN_OUT"] = str(out)
    subprocess.run([sys.executable, gen], check=True, env=env, capture_output=True)
    with open(os.path.join(root, "pquic_amd", "csrc", "bitslice_gen.h")) as f:
        assert out.read_text() == f.read()


def test_knobs_are_not_read_from_the_environment(lib):
    """The engine's kernel choices change only through fecgpu_set_knob: no FECGPU_* environment name
    is left in the library (the batching adapter's thread counts, PQUIC_FEC_BATCH_*, are its only
    environment settings), and a knob keeps its default whatever the environment holds."""
    data = open(LIB, "rb").read()
    names = set(re.findall(rb"FECGPU_[A-Z_]{3,}", data))
    assert not {n for n in names if not n.startswith((b"FECGPU_ERR", b"FECGPU_OK", b"FECGPU_BLOCK"))}, names
    v = C.c_int(-1)
    lib.fecgpu_get_knob.argtypes = [C.c_char_p, C.POINTER(C.c_int)]
    assert lib.fecgpu_get_knob(b"min_groups", C.byref(v)) == 0 and v.value == 1024
