"""Index sharding of one global RX batch over ranks: contiguous
shards, no exchange, conn table replicated.  Used by bench.py and the gloo tests."""
from __future__ import annotations


def shard_range(rank: int, world: int, n_per_rank: int):
    """[lo, hi) of the global frame indices owned by `rank` (weak scaling: fixed per-rank size)."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return rank * n_per_rank, (rank + 1) * n_per_rank


def split_range(rank: int, world: int, n_total: int):
    """[lo, hi) for a fixed global batch split as evenly as possible (strong scaling)."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return n_total * rank // world, n_total * (rank + 1) // world
