"""Does a block's repairs lying next to its sources in HBM help the decode apply?
The row-table entry points (fecgpu_rlc_encode_rows / fecgpu_rlc_decode_rows) take any layout, so the
same kernels run on two layouts of the headline's data (k16 r4 L1200, 2^20 blocks, 4 random erasures):
  separate  sources [b][16][L] and repairs [b][4][L] in two arrays (the bench's layout)
  combined  one array [b][20][L]: block b's 16 sources, then its 4 repairs
Encode (rows) and decode (rows: plan + apply, recovered rows in place) alternate over cycles; after
the timing every recovered row of both layouts must equal the original source.
usage: python tools/layout_probe.py [--cycles=N]"""
import ctypes as C
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import make_erasures  # noqa: E402
from pquic_amd import Engine  # noqa: E402

cycles = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--cycles=")), 5))
eng = Engine(0)
lib = eng.lib
v, u32, u64, sz = C.c_void_p, C.c_uint32, C.c_uint64, C.c_size_t
lib.fecgpu_rlc_encode_rows.argtypes = [v, v, u64, u32, u32, u32, u32, v, v]
dev = torch.device("cuda:0")
nb, k, r, L, e = 1 << 20, 16, 4, 1200, 4
src = torch.empty((nb, k, L), dtype=torch.uint8, device=dev)
eng.synth_fill(src, src.numel(), 0x5EEDF3C0, 0)
orig = src.clone()
rep = torch.empty((nb, r, L), dtype=torch.uint8, device=dev)
comb = torch.empty((nb, k + r, L), dtype=torch.uint8, device=dev)
comb[:, :k] = src
b = torch.arange(nb, device=dev, dtype=torch.int64).unsqueeze(1)
jk, jr = torch.arange(k, device=dev, dtype=torch.int64), torch.arange(r, device=dev, dtype=torch.int64)
tables = {
    "separate": (src.data_ptr() + (b * k + jk) * L, rep.data_ptr() + (b * r + jr) * L),
    "combined": (comb.data_ptr() + (b * (k + r) + jk) * L, comb.data_ptr() + (b * (k + r) + k + jr) * L),
}
tables = {n: (s.contiguous(), p.contiguous()) for n, (s, p) in tables.items()}
sp, miss = make_erasures(torch, nb, k, e, 11, dev)
rp = torch.zeros((nb, 2), dtype=torch.int64, device=dev)
rp[:, 0] = (1 << r) - 1
seeds = (((b & 0xFFFFFF) << 8) + jr).to(torch.int32).contiguous()  # the block framework's repair FPIDs
st = torch.empty(nb, dtype=torch.uint8, device=dev)
rec = torch.empty((nb, 2), dtype=torch.int64, device=dev)
ws = eng.alloc_workspace(nb, k, r)
stream = eng._stream(None)


def encode(name):
    s, p = tables[name]
    rc = lib.fecgpu_rlc_encode_rows(s.data_ptr(), p.data_ptr(), nb, k, r, L, 0, None, stream)
    assert rc == 0, rc


def decode(name):
    s, p = tables[name]
    rc = lib.fecgpu_rlc_decode_rows(s.data_ptr(), p.data_ptr(), nb, k, r, L, seeds.data_ptr(), sp.data_ptr(),
                                    rp.data_ptr(), st.data_ptr(), rec.data_ptr(), ws.data_ptr(), ws.numel(), stream)
    assert rc == 0, rc


ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
times = {}
for name in tables:  # warm
    encode(name)
    decode(name)
torch.cuda.synchronize()
for _ in range(cycles):
    for name in tables:
        for op, fn in (("encode", encode), ("decode", decode)):
            ev[0].record()
            for _ in range(3):
                fn(name)
            ev[1].record()
            torch.cuda.synchronize()
            times.setdefault((name, op), []).append(ev[0].elapsed_time(ev[1]) / 3)
# every recovered row equals the original: erase the rows, decode in place, compare
ms = miss.to(dev).sort(dim=1).values
rows = {"separate": (src.view(nb * k, L), (b * k + ms).reshape(-1)),
        "combined": (comb.view(nb * (k + r), L), (b * (k + r) + ms).reshape(-1))}
want = orig.view(nb * k, L)[(b * k + ms).reshape(-1)]
for name, (flat, idx) in rows.items():
    flat[idx] = 0xA5
    decode(name)
    torch.cuda.synchronize()
    okr = (st == 0).repeat_interleave(e)
    assert bool((flat[idx][okr] == want[okr]).all()), name
    print(f"{name}: {int((st == 0).sum())} blocks recovered, their rows equal to the originals", flush=True)
for (name, op), t in sorted(times.items(), key=lambda x: (x[0][1], x[0][0])):
    bytes_ = (k + r) * L * nb
    print(f"{op:6s} {name:9s} {statistics.median(t):7.3f} ms (min {min(t):.3f})  "
          f"{bytes_ / (statistics.median(t) * 1e-3) / 1e9:7.1f} GB/s of (k + r) L per block", flush=True)
