"""Index sharding of one global RX batch over ranks: contiguous
shards, no exchange, conn table replicated.  Used by bench.py and the gloo tests."""
from __future__ import annotations

import time


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


def common_window(body, dist=None):
    """Run body() inside one window shared by all ranks: the window opens when the start barrier
    releases this rank and closes after the end barrier, so every rank's window covers the slowest
    rank's finish.  Returns (max over ranks of the window, max over ranks of each rank's own
    body() time), both in seconds; dist = torch.distributed with an initialised group, or None for
    one process.  Ranks that ran one after another therefore cannot look parallel."""
    import torch

    multi = dist is not None and dist.is_initialized() and dist.get_world_size() > 1
    if multi:
        dist.barrier()
    t0 = time.perf_counter()
    body()
    t_own = time.perf_counter()
    if multi:
        dist.barrier()
    t1 = time.perf_counter()
    t = torch.tensor([t1 - t0, t_own - t0], dtype=torch.float64)
    if multi:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0]), float(t[1])
