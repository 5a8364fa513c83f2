"""The N>1 path on CPU: two gloo ranks shard the requests (istio_amd.dist.shard_bounds) and sum
their per-rule hit counters (istio_amd.dist.reduce_counters) -- the same calls bench.py makes over
RCCL.  Per-shard counters come from the oracle here (the GPU computes them with mxp_hits_device in
the -m gpu tests); the reduced counters must equal the whole batch's."""
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def test_shard_bounds_partition():
    from istio_amd.dist import shard_bounds
    for n in (0, 1, 7, 64, 1000, 1 << 20):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out_path):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    from istio_amd import dist as D
    from istio_amd import workloads as W
    manifest, rules, batch = W.c2_workload(n_rules=200, n_requests=3001, seed=5)
    lo, hi = D.shard_bounds(batch.n, rank, world)
    codes = oracle.oracle_matrix(oracle.OracleEvaluator(manifest), rules, batch, lo, hi, threads=2)
    hits = torch.from_numpy((codes == 1).sum(axis=0).astype(np.int64))
    D.reduce_counters(hits)
    slowest = D.max_over_ranks(float(rank + 1))
    if rank == 0:
        np.save(out_path, np.concatenate([hits.numpy(), [int(slowest)]]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_hit_counters(tmp_path):
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from istio_amd import workloads as W
    out = str(tmp_path / "hits.npy")
    mp.start_processes(_rank_main, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    got = np.load(out)
    manifest, rules, batch = W.c2_workload(n_rules=200, n_requests=3001, seed=5)
    want = (oracle.oracle_matrix(oracle.OracleEvaluator(manifest), rules, batch, threads=4) == 1).sum(axis=0)
    assert got[-1] == 2  # max over ranks of (rank + 1)
    assert np.array_equal(got[:-1], want) and want.sum() > 0
