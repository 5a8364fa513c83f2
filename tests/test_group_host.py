"""Host halves of the device-group C-ABI (include/mxp_group.h) that need no GPU: the shard layout
(mxp_group_shard_bounds) and the memquota key owners (mxp_group_key_owners) agree with the
torch.distributed harness's istio_amd/dist.py, the contiguous shard views partition a batch, and a
group refuses host-only members."""
import numpy as np
import pytest

from istio_amd import workloads as W


def test_shard_bounds_match_dist(libmxp):
    from istio_amd import dist as D
    from istio_amd.engine import shard_bounds
    for n in (0, 1, 7, 64, 1000, (1 << 20) + 3, 8 << 20):
        for w in (1, 2, 3, 8):
            assert [shard_bounds(n, k, w) for k in range(w)] == [D.shard_bounds(n, k, w) for k in range(w)]


def test_key_owners_match_dist(libmxp):
    """LPT over the C5 key shares (and ties: equal weights) -- the same owners as dist.key_owners."""
    from istio_amd import dist as D
    from istio_amd.engine import key_owners
    for K in (1, 16, 1024):
        for w in (W.quota_key_weights(K), np.ones(K), np.random.default_rng(K).random(K)):
            for n in (1, 2, 3, 8):
                assert np.array_equal(key_owners(w, n), D.key_owners(w, n)), (K, n)


def test_split_batch_partitions(libmxp):
    _, _, batch = W.c2_workload(n_rules=50, n_requests=1001, seed=2)
    parts = W.split_batch(batch, 3)
    assert [p.n for p in parts] == [334, 334, 333]
    for c in range(len(batch.names)):
        assert np.array_equal(np.concatenate([p.kinds[c] for p in parts]), batch.kinds[c])
        assert np.array_equal(np.concatenate([p.values[c] for p in parts]), batch.values[c])
        assert all(np.shares_memory(p.values[c], batch.values[c]) for p in parts)


def test_group_refuses_host_only_members(libmxp):
    from istio_amd.engine import Group, MxpError
    with pytest.raises(MxpError, match="groups need GPUs"):
        Group([-1])
