"""Engine against the CPU oracle on randomly drawn shapes (GPU suite).  The parametrized parity tests
in test_gpu_parity.py pick their shapes by hand; these draw k in 1..128, r in 1..min(128, ...), L a
multiple of 4 up to 9000 (the engine's rule, fecgpu.h), block counts from 1 up to a few thousand,
block numbers across the 24-bit wrap, and per block a random erasure count and repair subset
(sometimes too few repairs).  Encode bytes, decode statuses, recovered masks and recovered rows must
equal the oracle's, bit for bit; the packed apply (the bench's decode output) is checked against the
same rows.  Seeded: a failure names its case and reproduces."""
import numpy as np
import pytest

from oracle_py import Oracle, synth_bytes
import test_gpu_parity as parity
from test_gpu_parity import DEV, _run_decode_batch, bits, masks_from_lists, to_dev

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
CASES = 48


@pytest.fixture(scope="module")
def eng():
    from pquic_amd import Engine
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    return Engine(0)


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


def _shape(seed):
    rng = np.random.default_rng(0xF0220000 + seed)
    k = int(rng.choice([1, 2, 3, 4, 5, 8, 16, 30, 32, 64, 100, 128, int(rng.integers(1, 129))]))
    r = int(rng.choice([1, 2, 4, 8, 16, 32, int(rng.integers(1, 129))]))
    r = min(r, 128)
    L = 4 * int(rng.choice([1, 2, 16, 100, 300, 301, 512, 2250, int(rng.integers(1, 2251))]))
    nb = max(1, min(int(rng.choice([1, 3, 64, 257, 1000, 4100])), (16 << 20) // ((k + r) * L)))
    fbn_base = int(rng.choice([0, (1 << 24) - nb // 2 - 1, int(rng.integers(0, 1 << 24))])) & 0xFFFFFF
    return rng, k, r, L, nb, fbn_base


@pytest.mark.parametrize("seed", range(CASES))
def test_random_shape_encode_decode(eng, oracle, seed):
    rng, k, r, L, nb, fbn_base = _shape(seed)
    tag = f"seed {seed}: k {k} r {r} L {L} nb {nb} fbn_base {fbn_base:#x}"
    src_h = synth_bytes(nb * k * L, 0xC0DE + seed).reshape(nb, k, L)
    rep = torch.empty((nb, r, L), dtype=torch.uint8, device=DEV)
    eng.rlc_encode(to_dev(src_h), rep, k, r, L, fbn_base=fbn_base)
    torch.cuda.synchronize()
    rep_h = oracle.rlc_encode_batch(src_h, r, fbn_base)
    assert np.array_equal(rep.cpu().numpy(), rep_h), tag

    emax = min(k, r + 1)
    sp = np.zeros((nb, 2), np.uint64)
    rp = np.zeros((nb, 2), np.uint64)
    for b in range(nb):
        e = int(rng.integers(0, emax + 1))
        miss = set(rng.choice(k, e, replace=False).tolist())
        sp[b] = masks_from_lists(1, k, [[j for j in range(k) if j not in miss]])[0]
        nrep = int(rng.integers(max(0, e - 1), r + 1))
        rp[b] = masks_from_lists(1, r, [rng.choice(r, nrep, replace=False).tolist()])[0]
    work, got, st, rec = _run_decode_batch(eng, k, r, L, src_h, rep_h, sp, rp, fbn_base=fbn_base)
    ref = work.copy()
    st_ref, rec_ref = oracle.rlc_decode_batch(ref, rep_h, sp, rp, fbn_base)
    assert np.array_equal(st, st_ref), tag
    assert np.array_equal(rec, rec_ref), tag
    for b in range(nb):
        for j in bits(rec[b], k):
            assert np.array_equal(got[b, j], src_h[b, j]), (tag, b, j)
        for j in bits(sp[b], k):  # received sources are never touched
            assert np.array_equal(got[b, j], src_h[b, j]), (tag, b, j)

    # the bench's output form: plan, then the packed apply (row u of block b = its u-th erased source)
    w = to_dev(work)
    ws = eng.alloc_workspace(nb, k, r)
    eng.rlc_decode_plan(to_dev(sp), to_dev(rp), k, r, nb, ws, fbn_base=fbn_base)
    em = min(k, r)
    pk = torch.full((nb, em, L), 0x3C, dtype=torch.uint8, device=DEV)
    st2 = torch.full((nb,), 0xEE, dtype=torch.uint8, device=DEV)
    rec2 = torch.full((nb, 2), -1, dtype=torch.int64, device=DEV)
    eng.rlc_decode_apply_packed(w, to_dev(rep_h), pk, st2, rec2, k, r, L, nb, ws)
    torch.cuda.synchronize()
    assert np.array_equal(st2.cpu().numpy(), st_ref), tag
    assert np.array_equal(rec2.cpu().numpy().view(np.uint64), rec_ref), tag
    pk_h = pk.cpu().numpy()
    for b in range(nb):
        missing = [j for j in range(k) if j not in bits(sp[b], k)]
        for u, j in enumerate(missing[:em]):
            if j in bits(rec_ref[b], k):
                assert np.array_equal(pk_h[b, u], src_h[b, j]), (tag, b, j, "packed")


@pytest.mark.parametrize("seed", range(16))
@pytest.mark.parametrize("window_sc", [0, 2])
def test_random_window_encode(eng, oracle, seed, window_sc):
    """Sliding-window encode (window_framework_sender.h:214-250: block number 0, coefficients seeded
    by the repair index) on random (k, r, step, L, windows): overlapping, adjacent and gapped windows;
    window_sc 2 forces the shared-coefficient kernel (16-B-aligned L), 0 the block-at-a-time one."""
    rng = np.random.default_rng(0xF0230000 + seed)
    k = int(rng.integers(1, 65))
    r = int(rng.integers(1, 17))
    step = int(rng.integers(1, k + 8))
    L = 16 * int(rng.choice([1, 3, 75, 128, int(rng.integers(1, 565))]))
    nw = max(1, min(int(rng.integers(1, 600)), (8 << 20) // ((step + r) * L)))
    nsym = (nw - 1) * step + k
    sym_h = synth_bytes(nsym * L, 0xF1D0 + seed).reshape(nsym, L)
    rep = torch.empty((nw, r, L), dtype=torch.uint8, device=DEV)
    old = eng.get_knob("window_sc")
    try:
        eng.set_knob("window_sc", window_sc)
        eng.rlc_window_encode(to_dev(sym_h), rep, nw, step, k, r, L)
    finally:
        eng.set_knob("window_sc", old)
    torch.cuda.synchronize()
    got = rep.cpu().numpy()
    tag = f"seed {seed}: k {k} r {r} step {step} L {L} windows {nw} window_sc {window_sc}"
    for w in range(nw):
        want = oracle.rlc_encode_block(0, list(sym_h[w * step: w * step + k]), r)[1]
        for i in range(r):
            assert np.array_equal(got[w, i], want[i]), (tag, w, i)


@pytest.mark.parametrize("seed", range(16))
def test_random_xor(eng, oracle, seed):
    """XOR encode and single-erasure recover (xor_fec_scheme.c) on random k (the specialised kernels
    and the runtime-k one), L and block counts, erasures 0..2 per block, the repair sometimes absent."""
    rng = np.random.default_rng(0xF0240000 + seed)
    k = int(rng.choice([1, 2, 3, 4, 5, 6, 7, 8, 16, int(rng.integers(1, 129))]))
    L = 4 * int(rng.choice([1, 4, 300, 304, int(rng.integers(1, 2251))]))
    nb = max(1, min(int(rng.choice([1, 7, 100, 1000, 5000])), (16 << 20) // ((k + 1) * L)))
    src_h = synth_bytes(nb * k * L, 0xF2D0 + seed).reshape(nb, k, L)
    rep = torch.empty((nb, 1, L), dtype=torch.uint8, device=DEV)
    eng.xor_encode(to_dev(src_h), rep, k, L)
    torch.cuda.synchronize()
    rep_h = rep.cpu().numpy()
    tag = f"seed {seed}: k {k} L {L} nb {nb}"
    assert np.array_equal(rep_h, oracle.xor_encode_batch(src_h)), tag
    sp = np.zeros((nb, 2), np.uint64)
    rp = np.zeros((nb, 2), np.uint64)
    for b in range(nb):
        miss = set(rng.choice(k, min(int(rng.integers(0, 3)), k), replace=False).tolist())
        sp[b] = masks_from_lists(1, k, [[j for j in range(k) if j not in miss]])[0]
        rp[b] = masks_from_lists(1, 1, [[0]] if rng.random() < 0.8 else [[]])[0]
    work, got, st, rec = _run_decode_batch(eng, k, 1, L, src_h, rep_h, sp, rp, scheme="xor")
    ref = work.copy()
    st_ref, rec_ref = oracle.xor_decode_batch(ref, rep_h, sp, rp)
    assert np.array_equal(st, st_ref) and np.array_equal(rec, rec_ref), tag
    ok = st == 0
    assert np.array_equal(got[ok], src_h[ok]), tag


@pytest.mark.parametrize("seed", range(12))
def test_random_decode_rows(eng, oracle, seed):
    """The receive-side gather (fecgpu_rlc_decode_rows: every row anywhere in a shuffled pool, per-repair
    seeds, recovered rows written through the table) on random shapes: the parametrized parity test's
    body, with k, r, L and the block count drawn here."""
    rng = np.random.default_rng(0xF0250000 + seed)
    k = int(rng.integers(1, 129))
    r = int(rng.integers(1, 65))
    L = 4 * int(rng.choice([1, 5, 300, 304, int(rng.integers(1, 2251))]))
    nb = max(8, min(int(rng.choice([17, 300, 2000])), (8 << 20) // ((k + r) * L)))  # the body asserts some recovery
    parity.test_decode_rows_vs_oracle(eng, oracle, k, r, L, nb)  # through the module: not collected twice
