"""Multi-GPU plumbing for bench.py: one process per GPU, no data-path collective.

Verification shards by independent signatures: rank r verifies the
corpus slice [r*n, (r+1)*n) on its own device, weak scaling. The only collectives
are host-side gloo ones around the timed region (barrier, max of the elapsed time,
sum of failure flags); no RCCL/xGMI traffic is needed and none is invented.
"""
from __future__ import annotations

import time
from typing import Callable, Optional, Tuple


def shard_range(rank: int, world: int, per_rank: int) -> Tuple[int, int]:
    """Corpus indices owned by `rank` (weak scaling: `per_rank` items each)."""
    assert 0 <= rank < world and per_rank >= 0
    return rank * per_rank, (rank + 1) * per_rank


def timed_region(step: Callable[[], None], steps: int, sync: Callable[[], None], dist=None) -> float:
    """Barrier + sync, run `steps` steps, sync + barrier; return the MAX elapsed over ranks."""
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    return max_over_ranks(elapsed, dist)


def max_over_ranks(x: float, dist=None) -> float:
    if dist is None:
        return x
    import torch

    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_ranks_ok(ok: bool, dist=None) -> bool:
    if dist is None:
        return ok
    import torch

    t = torch.tensor([0 if ok else 1], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item()) == 0
