"""The value-class fill's two kernels (kernels.hip vtfill_imm_body): mxp_vtfill_imm<n>_kernel takes
the wave-tiles with no guard-kind errors, no class error words in the chunk and no error-plane
pairs, unrolled at compile time; it marks the rest (kargs.vtf_slow) for mxp_vtfill_imm_slow<n>_kernel.
Batches whose tiles split between the two -- continuation rules with lookup errors on a few
requests, a rule count whose last chunk is partial, a ragged request count -- give the same bitmaps,
error planes, compact flags and hit counters as the LDS-row fill (MXP_DEBUG_FLAGS 33554432, one
general kernel for every tile) and as value classes off, and match the oracle."""
import numpy as np
import pytest

import oracle
from istio_amd import workloads as W
from test_gpu_parity import compare

pytestmark = pytest.mark.gpu
FORCE, FORCE_LDS, OFF = "262144", str(262144 | 33554432), "131072"


@pytest.fixture(scope="module")
def mxp(libmxp):
    import istio_amd.engine as mxp
    return mxp


def engine_for(mxp, monkeypatch, flags, manifest, rules):
    monkeypatch.setenv("MXP_DEBUG_FLAGS", flags)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    return eng


@pytest.mark.parametrize("cont_frac", [0.02, 0.3])
def test_split_fill_device_identical(mxp, monkeypatch, cont_frac):
    import torch
    manifest, rules, batch = W.c4_workload(n_rules=1300, n_requests=40_000 + 3, seed=71, cont_frac=cont_frac)
    Wd = (len(rules) + 31) // 32
    out = []
    for flags in (FORCE, FORCE_LDS, OFF):
        eng = engine_for(mxp, monkeypatch, flags, manifest, rules)
        if flags != OFF:
            assert eng.ruleset_info()["value_class_columns"] >= 5
        db = eng.upload(batch)
        dm = torch.zeros((Wd, batch.n), dtype=torch.int32, device="cuda:0")
        de = torch.zeros_like(dm)
        cm = torch.zeros_like(dm)
        fl = torch.ones(batch.n, dtype=torch.uint8, device="cuda:0")
        hits = torch.zeros(len(rules), dtype=torch.int64, device="cuda:0")
        hc = torch.zeros_like(hits)
        for _ in range(2):
            db.eval_hits(dm.data_ptr(), de.data_ptr(), hits.data_ptr(), 0)
            db.eval_compact(cm.data_ptr(), fl.data_ptr(), hc.data_ptr(), 0)
        torch.cuda.synchronize()
        out.append([x.cpu().numpy() for x in (dm, de, hits, cm, fl, hc)])
        db.free()
        eng.close()
    for o in out[1:]:
        for a, b in zip(out[0], o):
            assert np.array_equal(a, b)
    fl = out[0][4]
    # a mix: some requests with errors (their tiles to the slow kernel), most without
    assert 0 < fl.sum() < batch.n and out[0][0].any()


def test_split_fill_oracle(mxp, monkeypatch):
    manifest, rules, batch = W.c4_workload(n_rules=1300, n_requests=6000 + 5, seed=72, cont_frac=0.05)
    eng = engine_for(mxp, monkeypatch, FORCE, manifest, rules)
    got, want = compare(eng, oracle.OracleEvaluator(manifest), rules, batch, sample_msgs=200)
    assert (want == 1).sum() > 1000 and (want >= 2).sum() > 0
