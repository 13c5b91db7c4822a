"""Multi-rank sharding (gloo, world_size 2): each rank encodes / decodes its own contiguous block
range with the global FEC block numbers; gathered results equal the single-rank run byte for
byte, and the max-over-ranks timing reduction used by bench.py works.
test_sharded_equals_single covers the sharding logic with the CPU oracle on each rank (CPU suite);
test_sharded_engine_ranks runs the device engine on each rank (two processes on one GPU, gpu
suite) over a range that crosses the 24-bit block-number wrap."""
import os
import socket
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, k, r, L, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch.distributed as dist
    from oracle_py import Oracle, synth_bytes
    from pquic_amd.shard import fbn_base_of, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    o = Oracle()
    b0, b1 = shard_range(total, world, rank)
    nb = b1 - b0
    src = synth_bytes(total * k * L, 99)[b0 * k * L: b1 * k * L].reshape(nb, k, L)
    rep = o.rlc_encode_batch(src, r, fbn_base_of(b0), 1)
    # decode with erasures of every 3rd source
    sp = np.zeros((nb, 2), np.uint64)
    rp = np.zeros((nb, 2), np.uint64)
    for b in range(nb):
        m = (1 << k) - 1
        for j in range((b0 + b) % 3, k, 3):
            if bin(((1 << k) - 1) & ~m).count("1") < r:
                m &= ~(1 << j)
        sp[b, 0] = m
        rp[b, 0] = (1 << r) - 1
    work = src.copy()
    st, rec = o.rlc_decode_batch(work, rep, sp, rp, fbn_base_of(b0), 1)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    parts = [None] * world
    dist.all_gather_object(parts, (b0, rep.tobytes(), st.tobytes(), work.tobytes()))
    if rank == 0:
        q.put((float(t.item()), parts))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_equals_single(world):
    import torch.multiprocessing as mp
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    from oracle_py import Oracle, synth_bytes
    total, k, r, L = 37, 8, 3, 64   # odd size: uneven shards
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(i, world, port, total, k, r, L, q)) for i in range(world)]
    for p in procs:
        p.start()
    tmax, parts = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == float(world)
    parts.sort(key=lambda x: x[0])
    rep = np.concatenate([np.frombuffer(p[1], np.uint8) for p in parts])
    o = Oracle()
    src = synth_bytes(total * k * L, 99).reshape(total, k, L)
    assert np.array_equal(rep, o.rlc_encode_batch(src, r, 0, 1).reshape(-1))
    work = np.concatenate([np.frombuffer(p[3], np.uint8) for p in parts]).reshape(total, k, L)
    st = np.concatenate([np.frombuffer(p[2], np.uint8) for p in parts])
    ok = st == 0
    assert ok.sum() > total * 0.8
    assert np.array_equal(work[ok], src[ok])


def test_shard_ranges_cover_exactly():
    sys.path.insert(0, ROOT)
    from pquic_amd.shard import shard_range, weak_range
    for total in (0, 1, 7, 1 << 20, (1 << 24) + 3):
        for world in (1, 2, 3, 8):
            rs = [shard_range(total, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1
    assert weak_range(1 << 20, 3) == (3 << 20, 4 << 20)


def _engine_worker(rank, world, port, g0, total, k, r, L, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch.distributed as dist
    from oracle_py import synth_bytes
    from pquic_amd import Engine
    from pquic_amd.shard import fbn_base_of, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = Engine(0)
    a, b = shard_range(total, world, rank)
    src_h = synth_bytes(total * k * L, 99)[a * k * L: b * k * L].reshape(b - a, k, L)
    src = torch.from_numpy(src_h).to("cuda:0")
    rep = torch.empty((b - a, r, L), dtype=torch.uint8, device="cuda:0")
    eng.rlc_encode(src, rep, k, r, L, fbn_base=fbn_base_of(g0 + a))
    torch.cuda.synchronize()
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    parts = [None] * world
    dist.all_gather_object(parts, (a, rep.cpu().numpy().tobytes()))
    if rank == 0:
        q.put((float(t.item()), parts))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_engine_ranks():
    """Two ranks (gloo; both on cuda:0) each run the device engine on their shard of a global range
    crossing block 2^24 with fbn_base_of(b0); the gathered repairs equal the oracle's unsharded
    encode of the whole range."""
    import torch.multiprocessing as mp
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    from oracle_py import Oracle, synth_bytes
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    world, g0, total, k, r, L = 2, (1 << 24) - 37, 75, 16, 4, 1200
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_engine_worker, args=(i, world, port, g0, total, k, r, L, q)) for i in range(world)]
    for p in procs:
        p.start()
    tmax, parts = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == float(world)
    parts.sort(key=lambda x: x[0])
    rep = np.concatenate([np.frombuffer(p[1], np.uint8) for p in parts])
    src = synth_bytes(total * k * L, 99).reshape(total, k, L)
    assert np.array_equal(rep, Oracle().rlc_encode_batch(src, r, g0 & 0xFFFFFF, 1).reshape(-1))
