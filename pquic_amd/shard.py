"""Block partitioning across GPUs.

FEC blocks are independent: a block never spans packets of another block and its decode
needs only its own symbols.  N GPUs therefore take contiguous block ranges and share
nothing on the data path; each rank derives its blocks' FEC block numbers from their
global indices, so every rank generates exactly the coefficients the single-GPU run would.
"""
from __future__ import annotations


def shard_range(nblocks_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [b0, b1) of `rank`; sizes differ by at most one block."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    q, rem = divmod(nblocks_total, world)
    b0 = rank * q + min(rank, rem)
    return b0, b0 + q + (1 if rank < rem else 0)


def fbn_base_of(global_block: int) -> int:
    """fec_block_number is a 24-bit field (plugins/fec/fec.h:44-50)."""
    return global_block & 0xFFFFFF


def weak_range(blocks_per_rank: int, rank: int) -> tuple[int, int]:
    """Weak scaling: every rank owns `blocks_per_rank` blocks of a global sequence."""
    return rank * blocks_per_rank, (rank + 1) * blocks_per_rank
