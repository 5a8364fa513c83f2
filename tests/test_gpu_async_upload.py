"""Asynchronous device packing (pack_device.cpp, round 5): mxp_batch_upload returns once the batch's
arrays are on the device and its first evaluation finishes the packing (value-class sizing, tables,
heads, dictionary); mxp_batch_upload_ex(MXP_UPLOAD_NO_WAIT) returns before the copies are in.  Batches
uploaded ahead of evaluations, and evaluated on a caller stream, give the same bitmaps as the
synchronous sequence."""
import numpy as np
import pytest
import torch

from istio_amd import workloads as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mxp(libmxp):
    import istio_amd.engine as mxp
    return mxp


def _bitmaps(db, n, R, stream):
    Wd = (R + 31) // 32
    dm = torch.empty((Wd, n), dtype=torch.int32, device="cuda")
    de = torch.empty((Wd, n), dtype=torch.int32, device="cuda")
    db.eval(dm.data_ptr(), de.data_ptr(), stream.cuda_stream)
    return dm, de


@pytest.mark.parametrize("kind", ["c2", "c4"])
def test_uploads_ahead_of_evaluations(mxp, kind):
    if kind == "c4":
        manifest, rules, batch = W.c4_workload(n_rules=1500, n_requests=120_000, seed=31)
    else:
        manifest, rules, batch = W.c2_workload(n_rules=1500, n_requests=120_000, seed=31)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    ref_m, ref_e = eng.eval_batch(batch)
    halves = [batch.subset(np.arange(0, 60_000)), batch.subset(np.arange(60_000, 120_000))]
    pinned = [mxp.pinned_batch(h) for h in halves]
    s = torch.cuda.Stream()
    for no_wait in (False, True):
        # both uploads first (the second one's copies beside the first one's packer), then both
        # evaluations on a caller stream, the second batch first
        dbs = [eng.upload(b, no_wait=no_wait) for b, _ in pinned]
        for db in dbs:
            db.wait_copied()
        outs = [None, None]
        for i in (1, 0):
            outs[i] = _bitmaps(dbs[i], 60_000, len(rules), s)
        torch.cuda.synchronize()
        for i in (0, 1):
            m = outs[i][0].cpu().numpy().view(np.uint32)
            e = outs[i][1].cpu().numpy().view(np.uint32)
            assert np.array_equal(m, ref_m[:, 60_000 * i:60_000 * (i + 1)]), (no_wait, i)
            assert np.array_equal(e, ref_e[:, 60_000 * i:60_000 * (i + 1)]), (no_wait, i)
        for db in dbs:
            db.free()
    for _, arena in pinned:
        arena.free()
    eng.close()


def test_free_before_evaluation(mxp):
    """A batch freed right after its upload (its packer possibly still running) recycles its blocks
    only after the packer: later uploads evaluate exactly."""
    manifest, rules, batch = W.c2_workload(n_rules=800, n_requests=80_000, seed=32)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    ref_m, _ = eng.eval_batch(batch)
    pb, arena = mxp.pinned_batch(batch)
    s = torch.cuda.Stream()
    for _ in range(4):
        eng.upload(pb, no_wait=True).free()
    db = eng.upload(pb)
    dm, _ = _bitmaps(db, batch.n, len(rules), s)
    torch.cuda.synchronize()
    assert np.array_equal(dm.cpu().numpy().view(np.uint32), ref_m)
    db.free()
    arena.free()
    eng.close()


@pytest.mark.parametrize("kind", ["c2", "c4"])
def test_failed_finish_pack_retried(mxp, monkeypatch, kind):
    """A device-packed batch whose packing finish fails at its first evaluation (injected after the
    value-class tables, MXP_DEBUG_FLAGS 1 << 29) stays unfinished: the evaluation reports the error,
    and the next evaluation of the same batch runs the whole finish again and gives the bitmaps of a
    batch that never failed (the batch used to be marked packed with half-built tables)."""
    if kind == "c4":
        manifest, rules, batch = W.c4_workload(n_rules=1500, n_requests=60_000, seed=33)
    else:
        manifest, rules, batch = W.c2_workload(n_rules=1500, n_requests=60_000, seed=33)
    ref = mxp.Engine(0)
    ref.set_vocabulary(manifest)
    ref.compile(rules)
    want_m, want_e = ref.eval_batch(batch)
    monkeypatch.setenv("MXP_DEBUG_FLAGS", str(1 << 29))
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    db = eng.upload(batch)
    s = torch.cuda.Stream()
    with pytest.raises(mxp.MxpError, match="injected finish_pack failure"):
        _bitmaps(db, batch.n, len(rules), s)
    dm, de = _bitmaps(db, batch.n, len(rules), s)
    torch.cuda.synchronize()
    assert np.array_equal(dm.cpu().numpy().view(np.uint32), want_m)
    assert np.array_equal(de.cpu().numpy().view(np.uint32), want_e)
    db.free()
