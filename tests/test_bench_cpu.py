"""bench.py's host logic on CPU (no GPU): the synthetic shards of a G-GPU run partition ONE seeded
batch (what configs[4]'s 8 x 1M requests are), and the group step makes exactly one reduction per step
after every member's evaluation and the memquota replay (a recording stand-in for the device group)."""
import os
import socket
import sys
import time

import numpy as np

import bench
from istio_amd import workloads as W


def _rows(batch):
    """Per request, every column's decoded value (string ids differ between batches)."""
    out = []
    for q in range(batch.n):
        row = []
        for c, name in enumerate(batch.names):
            k, v = int(batch.kinds[c][q]), int(batch.values[c][q])
            if k == 8:  # string map: its (key, value) strings
                a, b = int(batch.map_offsets[v]), int(batch.map_offsets[v + 1])
                v = tuple((batch.string(int(batch.map_keys[i])), batch.string(int(batch.map_values[i])))
                          for i in range(a, b))
            row.append((name, k, None if k == 0 else batch.string(v) if k in (1, 7, 9) else v))
        out.append(tuple(row))
    return out


def test_shards_partition_one_batch():
    args = bench.parse(["--requests", "300", "--rules", "64", "--fresh-steps", "1", "--gen-procs", "2"])
    data = bench.Data(args, 3, {"c2", "c4"})
    for kind in ("c2", "c4"):
        whole = (W.c2_workload(n_rules=64, n_requests=900 * 3, seed=2) if kind == "c2" else
                 W.c4_workload(n_rules=64, n_requests=900 * 3, seed=4))[2]
        for rep in range(3):  # the base set, then the two fresh sets: the next 900 requests each time
            shards = data.shards(kind, rep)
            assert [b.n for b in shards] == [300, 300, 300]
            got = sum((_rows(b) for b in shards), [])
            assert got == _rows(whole.subset(np.arange(rep * 900, rep * 900 + 900))), (kind, rep)


class _Rec:
    """Stand-in for istio_amd.engine.Group / GroupQuota recording the call order."""

    def __init__(self):
        self.calls = []

    def eval(self, *a):
        self.calls.append("quota" if len(a) == 2 and isinstance(a[1], int) else "eval")

    def reduce(self):
        self.calls.append("reduce")

    def sync(self):
        self.calls.append("sync")


def test_group_step_one_reduce_per_step():
    g = _Rec()
    now = [10**18]
    step = bench.group_step(g, object(), (g, object(), now), None)
    elapsed, ev = bench.timed_loop(step, 3, 2, 1, None, sync=g.sync, events=False)
    steps = [c for c in g.calls if c != "sync"]
    assert steps == ["eval", "quota", "reduce"] * 5 and ev == []
    assert now[0] == 10**18 + 5 * 10**8  # the quota clock advances one tick per step


def _launch_rank_main(rank, world, port, out_path):
    """bench.main's control flow under torch.distributed.run: rank 0 times the group's steps (a
    recording stand-in) while rank 1 waits at the closing barrier."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if rank == 0:
        g = _Rec()
        step = bench.group_step(g, object(), None, None)
        elapsed, _ = bench.timed_loop(step, 3, 1, 1, None, sync=g.sync, events=False)
        np.save(out_path, np.array([elapsed, len(g.calls)]))
    dist.barrier()
    dist.destroy_process_group()


def test_launch_rank0_times_alone():
    """Under the driver's N > 1 launch only rank 0 runs steps: its timing makes no collective the
    idle ranks would have to join (an all-reduce of the elapsed time deadlocked the rehearsed
    two-rank launch, profiles/r6_s23_launch_deadlock.log)."""
    import tempfile

    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    out = os.path.join(tempfile.mkdtemp(), "t.npy")
    ctx = mp.start_processes(_launch_rank_main, args=(2, port, out), nprocs=2, join=False, start_method="spawn")
    t0 = time.time()
    while not ctx.join(timeout=5):
        if time.time() - t0 > 90:
            for p in ctx.processes:
                p.terminate()
            raise AssertionError("the two-rank launch did not finish: a collective only rank 0 entered")
    got = np.load(out)
    assert got[1] >= 4  # warm-up + timed steps (eval + reduce each) and the syncs
