"""Index sharding of one global RX batch over ranks: contiguous
shards, no exchange, conn table replicated.  Used by bench.py and the gloo tests."""
from __future__ import annotations

import os
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


class ShmBarrier:
    """A barrier for the ranks of one node in a few microseconds (gloo's over TCP takes ~0.1-1 ms, which a
    20-step window of 0.5-ms steps would count): each rank publishes an epoch counter in its own 64-B cell
    of a shared-memory page and spins until every cell has reached the epoch.  No atomics: one writer per
    cell.  Set up collectively over `dist` (rank 0 creates the page, the name goes out by broadcast); a rank
    that never arrives makes the others fail after `timeout_s` instead of hanging."""

    def __init__(self, dist, rank: int, world: int, timeout_s: float = 120.0):
        import secrets
        from multiprocessing import shared_memory

        import numpy as np

        self.rank, self.world, self.timeout_s, self.epoch = rank, world, timeout_s, 0
        name = [f"pn_barrier_{secrets.token_hex(6)}" if rank == 0 else None]
        if rank == 0:
            self.shm = shared_memory.SharedMemory(name=name[0], create=True, size=64 * world)
        dist.broadcast_object_list(name, src=0)
        if rank != 0:
            self.shm = shared_memory.SharedMemory(name=name[0])
            # attaching registers the segment with this process's resource tracker too (Python < 3.13),
            # which would unlink it again at exit after rank 0 has: only the creator owns it
            from multiprocessing import resource_tracker

            resource_tracker.unregister(self.shm._name, "shared_memory")
        self.cells = np.ndarray((world, 8), dtype=np.int64, buffer=self.shm.buf)
        if rank == 0:
            self.cells[:] = 0
        dist.barrier()

    def __call__(self):
        self.epoch += 1
        self.cells[self.rank, 0] = self.epoch
        col = self.cells[:, 0]
        deadline = None
        spins = 0
        while col.min() < self.epoch:
            spins += 1
            if deadline is None:
                deadline = time.monotonic() + self.timeout_s
            elif time.monotonic() > deadline:
                raise TimeoutError(f"rank {self.rank}: shared-memory barrier {self.epoch} timed out")
            if spins > 256:  # past the first tens of microseconds: let an oversubscribed peer run
                os.sched_yield()

    def close(self, dist):
        dist.barrier()  # nobody reads the page any more
        del self.cells
        self.shm.close()
        if self.rank == 0:
            self.shm.unlink()


def common_window(body, dist=None, barrier=None):
    """Run body() inside one window shared by all ranks: the window opens when the start barrier
    releases this rank and closes after the end barrier, so every rank's window covers the slowest
    rank's finish.  Returns (max over ranks of the window, max over ranks of each rank's own
    body() time), both in seconds; dist = torch.distributed with an initialised group, or None for
    one process; barrier = the barrier to use (a ShmBarrier when the ranks share a node), default
    dist.barrier.  Ranks that ran one after another therefore cannot look parallel."""
    import torch

    multi = dist is not None and dist.is_initialized() and dist.get_world_size() > 1
    sync = barrier if barrier is not None else (dist.barrier if multi else None)
    if multi:
        sync()
    t0 = time.perf_counter()
    body()
    t_own = time.perf_counter()
    if multi:
        sync()
    t1 = time.perf_counter()
    t = torch.tensor([t1 - t0, t_own - t0], dtype=torch.float64)
    if multi:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0]), float(t[1])
