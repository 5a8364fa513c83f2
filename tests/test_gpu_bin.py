"""Recycled batch blocks (engine_impl.h BlockBin, mxp_batch_free): the bin stays under its cap when
batch sizes vary, a batch evaluated on a caller stream can be freed after that stream is destroyed
(the completion event is recorded by the evaluation itself), and results stay exact throughout."""
import ctypes

import numpy as np
import pytest
import torch

from istio_amd import workloads as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mxp(libmxp):
    import istio_amd.engine as mxp
    return mxp


def _bitmaps(eng, db, n, R):
    Wd = (R + 31) // 32
    dm = torch.empty((Wd, n), dtype=torch.int32, device="cuda")
    de = torch.empty((Wd, n), dtype=torch.int32, device="cuda")
    db.eval(dm.data_ptr(), de.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return dm.cpu().numpy().view(np.uint32), de.cpu().numpy().view(np.uint32)


def test_bin_cap_with_varying_batch_sizes(mxp, monkeypatch):
    monkeypatch.setenv("MXP_BIN_CAP_MB", "48")
    manifest, rules, batch = W.c2_workload(n_rules=400, n_requests=200_000, seed=11)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    ref_m, ref_e = eng.eval_batch(batch)
    sizes = [200_000, 7_000, 120_000, 31_000, 200_000, 2_000, 90_000, 200_000, 15_000, 160_000]
    keep = []
    for k, n in enumerate(sizes):
        sub = batch.subset(np.arange(n))
        db = eng.upload(sub)
        m, e = _bitmaps(eng, db, n, len(rules))
        assert np.array_equal(m, ref_m[:, :n]) and np.array_equal(e, ref_e[:, :n]), (k, n)
        keep.append(db)
        if len(keep) > 2:
            keep.pop(0).free()
        held, cap = eng.bin_stats()
        assert cap == 48 << 20 and held <= cap, (k, held, cap)
    while keep:
        keep.pop(0).free()
    assert eng.bin_stats()[0] <= 48 << 20


def test_free_after_caller_stream_destroyed(mxp):
    hip = ctypes.CDLL("libamdhip64.so.7")
    manifest, rules, batch = W.c2_workload(n_rules=300, n_requests=50_000, seed=12)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    ref_m, _ = eng.eval_batch(batch)
    Wd = (len(rules) + 31) // 32
    for _ in range(3):
        db = eng.upload(batch)
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        dm = torch.empty((Wd, batch.n), dtype=torch.int32, device="cuda")
        flags = torch.empty(batch.n, dtype=torch.uint8, device="cuda")
        db.eval_compact(dm.data_ptr(), flags.data_ptr(), 0, s.value)
        assert hip.hipStreamSynchronize(s) == 0
        assert hip.hipStreamDestroy(s) == 0
        db.free()  # records nothing on the destroyed stream
        assert np.array_equal(dm.cpu().numpy().view(np.uint32), ref_m)
    db = eng.upload(batch)  # draws the recycled blocks
    m, _ = _bitmaps(eng, db, batch.n, len(rules))
    assert np.array_equal(m, ref_m)
    db.free()
