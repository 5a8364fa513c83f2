"""Narrow batches (mxp_bag_batch2, mxp_batch_upload2): u32 values and offsets over the host link,
widened on the device.  A narrow upload evaluates bit for bit as the wide one (C2, C4 with string
maps, the fuzz family with INT64 / DOUBLE / DURATION / TIMESTAMP columns that stay wide), its Resolve
over the uploaded batch (batch = NULL: the engine's host view) equals the plain Resolve with error
texts, and a group takes narrow shards."""
import numpy as np
import pytest
import torch

from istio_amd import workloads as W
from istio_amd.bags import NarrowBatch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mxp(libmxp):
    import istio_amd.engine as mxp
    return mxp


def _bitmaps(db, n, R):
    Wd = (R + 31) // 32
    dm = torch.zeros((Wd, n), dtype=torch.int32, device="cuda")
    de = torch.zeros((Wd, n), dtype=torch.int32, device="cuda")
    db.eval(dm.data_ptr(), de.data_ptr(), 0)
    torch.cuda.synchronize()
    return dm.cpu().numpy(), de.cpu().numpy()


@pytest.mark.parametrize("wl", ["c2", "c4", "fuzz"])
def test_narrow_upload_bit_identical(mxp, wl):
    if wl == "c2":
        manifest, rules, batch = W.c2_workload(n_rules=2000, n_requests=150_001, seed=81)
    elif wl == "c4":
        manifest, rules, batch = W.c4_workload(n_rules=2000, n_requests=150_001, seed=82)
    else:
        manifest = W.DEFAULT_TEST_MANIFEST
        rules = W.fuzz_rules(600, seed=83, depth=3)
        from istio_amd.bags import BagBatch
        batch = BagBatch.from_bags(W.fuzz_bags(4001, seed=84, p_wrong=0.0), names=list(manifest))
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    st = eng.compile(rules)
    rules_ok = [r for r, s in zip(rules, st) if s == 0]
    if len(rules_ok) != len(rules):
        eng.compile(rules_ok)
    nb = NarrowBatch(batch)
    if wl == "fuzz":
        assert 0 < int(nb.narrow.sum()) < len(batch.names)  # (numeric columns stay wide)
    else:
        assert nb.narrow.all() and nb.wire_bytes() < 0.8 * sum(
            a.nbytes for a in list(batch.kinds) + list(batch.values) + [batch.str_blob, batch.str_offsets,
                                                                          batch.map_offsets, batch.map_keys,
                                                                          batch.map_values])
    want = _bitmaps(eng.upload(batch), batch.n, len(rules_ok))
    for no_wait in (False, True):
        db = eng.upload2(nb, no_wait=no_wait)
        got = _bitmaps(db, batch.n, len(rules_ok))
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1]), no_wait
        db.free()
    assert want[0].any()


def test_narrow_resolve_uploaded(mxp):
    manifest, _, _ = W.c2_workload(n_rules=1500, n_requests=1, seed=2)
    rules = W.c2_rules(1500, seed=2)[0]
    R = len(rules)
    ns, vm, z = ["istio-system"] * R, np.ones(R, dtype=np.uint32), np.zeros(R, dtype=np.uint8)
    batches = [W.c2_workload(n_rules=1500, n_requests=3 * 70_001, seed=2, shard=(k * 70_001, (k + 1) * 70_001))[2]
               for k in range(3)]
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    eng.set_resolver("destination.service", "istio-system", ns, vm, z, z)
    want, texts = [], []
    for b in batches:
        w = eng.resolve_arrays(b, 0, ids16=True)
        want.append(w)
        err = np.nonzero(w[0] == 3)[0][:30]
        texts.append([eng.pair_error(int(q), int(w[1][q])) for q in err])
    narrow = [mxp.pinned_narrow(b) for b in batches]
    nxt = eng.upload2(narrow[0][0], no_wait=True)
    for k in range(3):
        cur = nxt
        if k + 1 < 3:
            nxt = eng.upload2(narrow[k + 1][0], no_wait=True)
        got = eng.resolve_uploaded(cur, 0, cap=1 << 22, ids16=True)
        for a, c in zip(got, want[k]):
            assert np.array_equal(a, c), k
        err = np.nonzero(want[k][0] == 3)[0][:30]
        assert [eng.pair_error(int(q), int(got[1][q])) for q in err] == texts[k]
    assert sum(len(t) for t in texts) > 0
    g = mxp.Group([0, 0])
    g.set_vocabulary(manifest)
    g.compile(rules)
    g.set_resolver("destination.service", "istio-system", ns, vm, z, z)
    for k in range(3):
        shards = [NarrowBatch(s) for s in W.split_batch(batches[k], 2)]
        gb = g.upload2(shards)
        got = g.resolve_arrays(None, 0, cap=1 << 22, ids16=True, uploaded=gb)
        for a, c in zip(got, want[k]):
            assert np.array_equal(a, c), k


def test_narrow_malformed_batches_rejected(mxp):
    """The u32 checks of a narrow upload (check_batch on the narrow arrays, no widened host copy)
    reject every malformed variant of test_batch_check.py with the same messages the wide upload
    gives, and the engine then uploads and evaluates the good batch as the wide path does."""
    import test_batch_check as T
    eng = mxp.Engine(0)
    eng.set_vocabulary(T.MANIFEST)
    assert (eng.compile(T.RULES) == 0).all()
    b = T.good_batch()
    n_maps = len(b.map_offsets) - 1
    cases = []
    for label, frag, x in T.malformed(b):
        if label == "map id":  # (1 << 40 is no u32: the first id past the map table instead)
            x.values[T._col(x, "ar")][5] = n_maps
        cases.append((label, frag, x))
    assert len(cases) == 9
    for label, frag, x in cases:
        with pytest.raises(mxp.MxpError) as ei:
            eng.upload2(NarrowBatch(x))
        msg = str(ei.value)
        assert "failed (1)" in msg and frag in msg, (label, msg)
        with pytest.raises(mxp.MxpError) as ei:  # (the same text from the wide upload)
            eng.upload(x)
        assert frag in str(ei.value), label
    R, n = len(T.RULES), b.n
    m_narrow, e_narrow = _bitmaps(eng.upload2(NarrowBatch(b)), n, R)
    m_wide, e_wide = _bitmaps(eng.upload(b), n, R)
    assert np.array_equal(m_narrow, m_wide) and np.array_equal(e_narrow, e_wide)
