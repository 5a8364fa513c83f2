"""Multi-GPU plumbing of the engine.

* Requests shard across ranks and the compiled rule / DFA / list tables are replicated: a Check
  request's predicates read only its own bag and the immutable rule set (resolver.go:202-238).
* memquota keys have ONE owner rank each (`key_owners`, balanced by expected load): the quota
  requests of a key are routed to its owner, so each key's arrival sequence is replayed on one GPU
  exactly as memquota.go:118-211 replays it in one process.  The per-key state never has to move.
* The only exchange is one sum all-reduce per step over the concatenated per-step counters
  `hits[R] ++ quota_delta[K]` (`StepCounters`), RCCL over xGMI ("nccl" backend on ROCm), "gloo" in
  the CPU tests.
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


def key_owners(weights, world_size: int):
    """Owner rank of every memquota key (one owner per key: the rank that holds the key's cell /
    rolling window and replays all of its requests in arrival order), assigned by expected load:
    longest-processing-time first over the keys' request frequencies at snapshot time (`weights`,
    e.g. the last batch's per-key counts), each key to the least-loaded rank, ties by rank then key.
    Greedy LPT is within 4/3 of the best assignment; a key whose own share exceeds 1/world bounds any
    one-owner assignment (C5's Zipf(1.05) head key: 15.5% of the requests, 1.24x the mean at 8 ranks)."""
    import heapq

    import numpy as np
    w = np.asarray(weights, dtype=np.float64)
    owners = np.zeros(len(w), dtype=np.int64)
    load = [(0.0, r) for r in range(world_size)]
    for k in np.lexsort((np.arange(len(w)), -w)):  # heaviest first, then by key id
        l, r = heapq.heappop(load)
        owners[k] = r
        heapq.heappush(load, (l + float(w[k]), r))
    return owners


def _initialized() -> bool:
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def reduce_counters(t):
    """Sum a counter tensor over all ranks, in place (no-op on a single process)."""
    import torch.distributed as dist
    if _initialized():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


class StepCounters:
    """Per-step counters reduced with ONE collective per step.

    Layout: one int64 tensor = the concatenation of `sizes` (e.g. hits[R] ++ quota_delta[K]).  The
    kernels of a step ACCUMULATE into `views()` (fused hit counters, memquota deltas); `end_step()`
    all-reduces that step's buffer and adds it to the running `total`.  On a single process the step
    buffer IS the total and nothing is reduced -- no extra work in the timed region.  With several
    ranks the step buffer is zeroed by `begin_step()`, so each step reduces only that step's counts
    (reducing a cumulative buffer every step would re-add the other ranks' earlier totals).
    """

    def __init__(self, sizes, device=None):
        import torch
        self.sizes = list(sizes)
        self.multi = _initialized()
        self.total = torch.zeros(sum(self.sizes), dtype=torch.int64, device=device)
        self.step = torch.zeros_like(self.total) if self.multi else self.total

    def views(self):
        """The step buffer split per counter family (views share its storage)."""
        return list(self.step.split(self.sizes))

    def totals(self):
        return list(self.total.split(self.sizes))

    def begin_step(self):
        if self.multi:
            self.step.zero_()

    def end_step(self):
        if self.multi:
            reduce_counters(self.step)  # the step's single collective
            self.total.add_(self.step)


def max_over_ranks(x: float, device=None) -> float:
    """Max of a scalar over ranks (the bench's step time is the slowest rank's)."""
    import torch
    import torch.distributed as dist
    if not _initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, device=None) -> float:
    """Sum of a scalar over ranks (e.g. the quota requests each owner rank received)."""
    import torch
    import torch.distributed as dist
    if not _initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
