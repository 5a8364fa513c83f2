"""bench.py's host logic on CPU (no GPU): the synthetic shards of a G-GPU run partition ONE seeded
batch (what configs[4]'s 8 x 1M requests are), and the group step makes exactly one reduction per step
after every member's evaluation and the memquota replay (a recording stand-in for the device group)."""
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
