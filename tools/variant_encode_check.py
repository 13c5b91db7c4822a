"""Encode bytes of A/B library builds against the in-tree one (tools/lib_ab.py --check covers the decode
apply only): k16 r4, k32 r8 (2^16 blocks, 1200 B) and k64 r16 (2^10 blocks, 9000 B) repairs of the same
synthetic sources must be byte-equal.
usage (GPU box): python tools/variant_encode_check.py path.so ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pquic_amd import Engine  # noqa: E402

dev = torch.device("cuda:0")
head = Engine(0)
rc = 0
for path in sys.argv[1:]:
    eng = Engine(0, lib_path=path)
    for k, r, L, nb in ((16, 4, 1200, 1 << 16), (32, 8, 1200, 1 << 16), (64, 16, 9000, 1 << 10)):
        src = torch.empty(nb * k * L, dtype=torch.uint8, device=dev)
        head.synth_fill(src, src.numel(), seed=k * 1000 + r)
        want = torch.zeros(nb * r * L, dtype=torch.uint8, device=dev)
        got = torch.full_like(want, 0x5A)
        head.rlc_encode(src, want, k, r, L)
        eng.rlc_encode(src, got, k, r, L)
        torch.cuda.synchronize()
        ok = bool(torch.equal(want, got))
        rc |= not ok
        print(f"{path}: k{k} r{r} L{L} x {nb}: {'equal' if ok else 'DIFFERENT'}", flush=True)
sys.exit(rc)
