"""The sharding semantics of the N>1 path on CPU, as separate processes: two gloo ranks shard the
requests (istio_amd.dist.shard_bounds, = mxp_group_shard_bounds) and sum their per-rule hit counters
(istio_amd.dist.reduce_counters); memquota keys owned by one rank each (dist.key_owners, =
mxp_group_key_owners) replay exactly the single-process sequence.  The product's device group
(include/mxp_group.h) does the same inside one process, with one RCCL all-reduce per step.  Per-shard counters come from the oracle here (the GPU computes them with mxp_hits_device in
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


def _step_rank_main(rank, world, port, out_path, steps):
    """bench.py's step structure with engine-free kernels: each step accumulates into the step views
    of StepCounters (hits[R] ++ quota_delta[K]) and ends with the step's single all-reduce."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import memquota as M
    from istio_amd import dist as D
    from istio_amd import workloads as W
    R, K = 37, 16
    calls = []
    orig = D.reduce_counters

    def counting_reduce(t):
        calls.append(t.numel())
        return orig(t)
    D.reduce_counters = counting_reduce
    ctr = D.StepCounters([R, K])
    # memquota requests routed by key owner: the rank replays its keys' sequences with the oracle
    mx, vd, keys, amounts, be, idx = W.quota_workload(n_keys=K, n_requests=400, seed=9, rank=rank, world=world,
                                                      return_index=True)
    assert np.all(D.key_owners(W.quota_key_weights(K), world)[keys] == rank)
    mq = M.Memquota({k: (int(mx[k]), int(vd[k])) for k in range(K)})
    granted_all = []
    for s in range(steps):
        ctr.begin_step()
        hits, delta = ctr.views()
        hits += torch.arange(R, dtype=torch.int64) * (rank + 1) + s  # a "kernel" accumulating into the step
        granted = [mq.handle(int(k), int(a), bool(b), 10**18 + s * 10**8) for k, a, b in zip(keys, amounts, be)]
        for k, g in zip(keys, granted):
            delta[int(k)] += g
        granted_all.append(granted)
        ctr.end_step()
    h, d = ctr.totals()
    if rank == 0:
        np.save(out_path, np.concatenate([h.numpy(), d.numpy(), [len(calls)]]))
    np.save(out_path + ".r%d.npy" % rank, np.concatenate([idx, np.array(granted_all).reshape(-1)]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_step_counters_and_quota_owners(tmp_path):
    """bench.py's step at world_size 2: per-step buffers reduced once per step (totals are exact after
    several steps -- no re-adding of earlier totals), and memquota requests routed to their key's
    owner rank reproduce the single-process sequential HandleQuota exactly."""
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import memquota as M
    from istio_amd import workloads as W
    out = str(tmp_path / "ctr.npy")
    steps, world, R, K = 3, 2, 37, 16
    mp.start_processes(_step_rank_main, args=(world, _free_port(), out, steps), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(out)
    want_hits = sum(np.arange(R) * (r + 1) + s for r in range(world) for s in range(steps))
    assert np.array_equal(got[:R], want_hits)
    assert got[-1] == steps  # one collective per step
    # single process: the whole arrival stream (n_requests * world requests, same draw), sequentially
    mx, vd, keys, amounts, be = W.quota_workload(n_keys=K, n_requests=400 * world, seed=9)
    mq = M.Memquota({k: (int(mx[k]), int(vd[k])) for k in range(K)})
    want_delta = np.zeros(K, dtype=np.int64)
    want_granted = np.zeros((steps, len(keys)), dtype=np.int64)
    for s in range(steps):
        for i, (k, a, b) in enumerate(zip(keys, amounts, be)):
            g = mq.handle(int(k), int(a), bool(b), 10**18 + s * 10**8)
            want_granted[s, i] = g
            want_delta[int(k)] += g
    assert np.array_equal(got[R:R + K], want_delta)
    for r in range(world):
        v = np.load(out + ".r%d.npy" % r)
        n = (len(v)) // (steps + 1)
        idx, granted = v[:n], v[n:].reshape(steps, n)
        assert np.array_equal(granted, want_granted[:, idx])


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


def _quota_rank_main(rank, world, port, out_path, n_keys, per_rank):
    """One step of C5's quota half at world 8: the rank replays the requests of the keys it owns
    (dist.key_owners, LPT by expected load) with the memquota restatement, its per-key deltas and its
    request count go through one all-reduce each."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import memquota as M
    from istio_amd import dist as D
    from istio_amd import workloads as W
    mx, vd, keys, amounts, be = W.quota_workload(n_keys=n_keys, n_requests=per_rank, seed=11, rank=rank, world=world)
    mq = M.Memquota({k: (int(mx[k]), int(vd[k])) for k in range(n_keys)})
    ctr = D.StepCounters([n_keys, world])
    ctr.begin_step()
    delta, count = ctr.views()
    for k, a, b in zip(keys, amounts, be):
        delta[int(k)] += mq.handle(int(k), int(a), bool(b), 10**18)
    count[rank] = len(keys)
    ctr.end_step()
    if rank == 0:
        np.save(out_path, np.concatenate([t.numpy() for t in ctr.totals()]))
    dist.barrier()
    dist.destroy_process_group()


def test_eight_rank_quota_owners_balanced(tmp_path):
    """configs[4]'s quota routing at 8 ranks: keys owned by load (LPT over the Zipf(1.05) key shares)
    put at most 1.25x the mean on a rank -- the head key's own 15.5% share bounds any one-owner
    assignment at 1.24x (key % 8 gave 1.9x) -- and the all-reduced deltas equal the single-process
    sequential HandleQuota (memquota.go:118-211)."""
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import memquota as M
    from istio_amd import dist as D
    from istio_amd import workloads as W
    world, K, per_rank = 8, 1024, 6000
    owners = D.key_owners(W.quota_key_weights(K), world)
    load = np.bincount(owners, weights=W.quota_key_weights(K), minlength=world)
    assert load.max() * world <= 1.25 and load.max() * world < np.bincount(np.arange(K) % world, weights=W.quota_key_weights(K)).max() * world
    out = str(tmp_path / "q.npy")
    mp.start_processes(_quota_rank_main, args=(world, _free_port(), out, K, per_rank), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(out)
    counts = got[K:]
    assert counts.sum() == world * per_rank and counts.max() <= 1.25 * counts.mean(), counts
    mx, vd, keys, amounts, be = W.quota_workload(n_keys=K, n_requests=per_rank * world, seed=11)
    mq = M.Memquota({k: (int(mx[k]), int(vd[k])) for k in range(K)})
    want = np.zeros(K, dtype=np.int64)
    for k, a, b in zip(keys, amounts, be):
        want[int(k)] += mq.handle(int(k), int(a), bool(b), 10**18)
    assert np.array_equal(got[:K], want)
