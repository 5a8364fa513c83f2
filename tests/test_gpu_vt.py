"""Value classes (kernels.hip mxp_vt_*): rules that read one column as a string are evaluated once per
distinct value of that column in the batch and their words gathered per request.  Bar: bit-exact
against the oracle (and against the engine with value classes off), error texts included -- the
class records the class kernel logs at a representative request are expanded to every request of
the class (engine.cpp expand_class_errors).  MXP_DEBUG_FLAGS 262144 forces value classes at any
batch size (the default wants >= 16 requests per class); 131072 turns them off; 2097152 makes the
fill chunks gather class words from global memory instead of the LDS-staged rows
(mxp_vtfill_kernel vs mxp_vtfill_lds_kernel); 33554432 keeps batches whose class tables all have 64
slots on mxp_vtfill_lds_kernel instead of mxp_vtfill_imm<n>_kernel."""
import numpy as np
import pytest

import oracle
from istio_amd import workloads as W
from istio_amd.bags import BagBatch
from test_gpu_parity import compare

pytestmark = pytest.mark.gpu
FORCE, OFF, GLOBAL = "262144", "131072", "2097152"
FORCE_GLOBAL = str(262144 | 2097152)
FORCE_LDS = str(262144 | 33554432)  # the LDS-row kernel instead of the immediate-offset one (tables of 64 slots)


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


@pytest.mark.parametrize("flags", [FORCE, "0", FORCE_GLOBAL, FORCE_LDS])
def test_c4_value_classes_parity(mxp, monkeypatch, flags):
    """C4 routes: the header rules (equality and regexps on request.headers["h"]) become value
    classes (17 values per header); path rules stay with the prefix index."""
    manifest, rules, batch = W.c4_workload(n_rules=600, n_requests=3000, seed=44)
    eng = engine_for(mxp, monkeypatch, flags, manifest, rules)
    assert eng.ruleset_info()["value_class_columns"] >= 5
    got, want = compare(eng, oracle.OracleEvaluator(manifest), rules, batch)
    assert (want == 1).sum() > 1000


@pytest.mark.parametrize("flags", [FORCE, FORCE_LDS])
def test_fuzz_value_classes_errors(mxp, monkeypatch, flags):
    """Random rules over random bags with missing / wrongly typed values: class records (lookup and
    conversion errors, panics) expanded to every request of the class, texts checked; class words
    with error bits (the immediate-offset kernel's global error gathers)."""
    rules = W.fuzz_rules(800, seed=61, depth=3)
    batch = BagBatch.from_bags(W.fuzz_bags(900, seed=62), names=list(W.DEFAULT_TEST_MANIFEST))
    eng = engine_for(mxp, monkeypatch, flags, W.DEFAULT_TEST_MANIFEST, rules)
    assert eng.ruleset_info()["value_class_columns"] >= 1
    got, want = compare(eng, oracle.OracleEvaluator(W.DEFAULT_TEST_MANIFEST), rules, batch, sample_msgs=800)
    assert (want >= 2).sum() > 100


def test_guarded_fuzz_value_classes(mxp, monkeypatch):
    rules = W.guarded_fuzz_rules(1500, seed=63)
    batch = BagBatch.from_bags(W.fuzz_bags(3000 + 29, seed=64), names=list(W.DEFAULT_TEST_MANIFEST))
    eng = engine_for(mxp, monkeypatch, FORCE, W.DEFAULT_TEST_MANIFEST, rules)
    compare(eng, oracle.OracleEvaluator(W.DEFAULT_TEST_MANIFEST), rules, batch)


def test_value_classes_on_off_identical_with_hits(mxp, monkeypatch):
    """Device path (bitmaps + fused / streamed hit counters): value classes on (class words from
    LDS-staged rows, or gathered from global memory) and off agree; a ragged batch ends inside a
    staged workgroup's tiles."""
    import torch
    manifest, rules, batch = W.c4_workload(n_rules=2000, n_requests=50_000 + 5, seed=45)
    out = []
    for flags in (FORCE, FORCE_GLOBAL, OFF, FORCE_LDS):
        eng = engine_for(mxp, monkeypatch, flags, manifest, rules)
        db = eng.upload(batch)
        Wd = (len(rules) + 31) // 32
        dm = torch.zeros((Wd, batch.n), dtype=torch.int32, device="cuda:0")
        de = torch.zeros_like(dm)
        hits = torch.zeros(len(rules), dtype=torch.int64, device="cuda:0")
        for _ in range(3):  # the fused / streaming choice follows the previous evaluation
            db.eval_hits(dm.data_ptr(), de.data_ptr(), hits.data_ptr(), 0)
        torch.cuda.synchronize()
        out.append((dm.cpu().numpy(), de.cpu().numpy(), hits.cpu().numpy()))
        db.free()
    for o in out[1:]:
        assert np.array_equal(out[0][0], o[0]) and np.array_equal(out[0][1], o[1])
        assert np.array_equal(out[0][2], o[2])
    assert out[0][2].sum() > 0


def test_resolver_with_value_classes(mxp, monkeypatch):
    """mxp_resolve_batch with value classes forced equals the run without them (selected rules,
    statuses, first-error rules and their texts)."""
    res = []
    for flags in (FORCE, FORCE_GLOBAL, OFF):
        manifest, rules, conf, batch = W.resolver_workload(n_rules=500, n_requests=2000, seed=65)
        eng = engine_for(mxp, monkeypatch, flags, manifest, rules)
        eng.set_resolver(**conf)
        status, err_rule, sel = eng.resolve(batch, 1)
        texts = [eng.pair_error(int(q), int(err_rule[q])) for q in np.nonzero(status == 3)[0]]
        res.append((status, err_rule[status == 3], [s.tolist() for s in sel], texts))
    assert np.array_equal(res[0][0], res[1][0]) and np.array_equal(res[0][1], res[1][1])
    assert res[0][2] == res[1][2] and res[0][3] == res[1][3]


@pytest.mark.parametrize("cap", ["1", "50"])
def test_value_class_records_past_capacity(mxp, monkeypatch, cap):
    """Class records whose expansion overflows the log: the rest come from recomputed windows."""
    monkeypatch.setenv("MXP_ERRCAP", cap)
    rules = W.fuzz_rules(300, seed=66, depth=2)
    batch = BagBatch.from_bags(W.fuzz_bags(600, seed=67), names=list(W.DEFAULT_TEST_MANIFEST))
    eng = engine_for(mxp, monkeypatch, FORCE, W.DEFAULT_TEST_MANIFEST, rules)
    compare(eng, oracle.OracleEvaluator(W.DEFAULT_TEST_MANIFEST), rules, batch, sample_msgs=300)
