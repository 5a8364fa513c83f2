"""Batch packing on the host (mxp_batch_pack_host, the host half of mxp_batch_upload): interning of
batch strings against the rule set's pools and the per-batch overlay, with parallel hash-sharded
deduplication.  Host-only engine: no GPU needed."""
import numpy as np
import pytest

from istio_amd import workloads as W
from istio_amd.bags import BYTES, STRING, BagBatch


@pytest.fixture(scope="module")
def Engine(libmxp):
    from istio_amd.engine import Engine
    return Engine


def doubled_table(b: BagBatch) -> BagBatch:
    """The same bags with a string table holding every string twice; odd requests (and every map)
    point at the second copy.  Interning must see through the duplicates."""
    ns = len(b.str_offsets) - 1
    end = int(b.str_offsets[-1])
    blob = np.concatenate([b.str_blob[:end], b.str_blob[:end], np.zeros(1, np.uint8)])
    offs = np.concatenate([b.str_offsets[:-1], b.str_offsets + np.uint64(end)])
    vals = []
    odd = (np.arange(b.n) % 2) == 1
    for k, v in zip(b.kinds, b.values):
        v = v.copy()
        sel = odd & ((k == STRING) | (k == BYTES))
        v[sel] += np.uint64(ns)
        vals.append(v)
    return BagBatch(b.n, b.names, b.kinds, vals, blob, offs, b.time_sec, b.time_nsec, b.map_offsets,
                    b.map_keys + np.uint32(ns), b.map_values + np.uint32(ns))


@pytest.mark.parametrize("family", ["c2", "fuzz", "c4"])
def test_pack_dedupes_duplicate_strings(Engine, family):
    if family == "c2":
        manifest, rules, batch = W.c2_workload(n_rules=500, n_requests=20000, seed=5)
    elif family == "c4":
        manifest, rules, batch = W.c4_workload(n_rules=300, n_requests=3000, seed=4)
    else:
        manifest = W.DEFAULT_TEST_MANIFEST
        rules = W.guarded_fuzz_rules(600, seed=43)
        batch = BagBatch.from_bags(W.fuzz_bags(3000, seed=44), names=list(manifest))
    eng = Engine(-1)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    one = eng.pack_host(batch)
    two = eng.pack_host(doubled_table(batch))
    assert one == two
    assert one["overlay_strings"] > 0
    if family == "c2":
        # source.ip bytes: one overlay entry per distinct address outside the rule set
        ips = {bytes(batch.str_blob[int(batch.str_offsets[v]):int(batch.str_offsets[v + 1])])
               for k, v in zip(batch.kinds[batch.names.index("source.ip")], batch.values[batch.names.index("source.ip")])
               if k == BYTES}
        assert 0 < one["overlay_bytes"] <= len(ips)


def test_pack_requires_rules(Engine):
    eng = Engine(-1)
    eng.set_vocabulary(W.DEFAULT_TEST_MANIFEST)
    with pytest.raises(Exception):
        eng.pack_host(BagBatch.from_bags([{}], names=list(W.DEFAULT_TEST_MANIFEST)))
