"""Multi-GPU plumbing of the engine: requests shard across ranks, rule tables are replicated, and the
only exchange is a sum all-reduce of per-rule counters (hit counters; later memquota deltas) --
SURVEY.md 8(e).  One process per GPU under torch.distributed (backend "nccl" = RCCL over xGMI on
ROCm; "gloo" in the CPU tests).
"""
from __future__ import annotations

import os


def world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_bounds(n_total: int, rank: int, world_size: int) -> tuple[int, int]:
    """Contiguous request shard [lo, hi) of `rank`: sizes differ by at most one request."""
    base, extra = divmod(n_total, world_size)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def reduce_counters(t):
    """Sum a per-rule counter tensor over all ranks, in place (no-op on a single process)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def max_over_ranks(x: float, device=None) -> float:
    """Max of a scalar over ranks (the bench's step time is the slowest rank's)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
