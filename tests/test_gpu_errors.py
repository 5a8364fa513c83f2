"""Error records past the log's capacity (MXP_ERRCAP): the error bits are the truth and the records a
cache -- a pair whose bit is set but whose record did not fit is re-evaluated on demand (its window of
requests, mxp_engine::recompute_errors), so mxp_pair_error / resolver PRED_ERROR texts never come back
empty for a failing pair.  Reference: resolver.go:225-227 (first predicate error fails the Resolve),
grpcServer.go:160-163 (INTERNAL with that error's text)."""
import numpy as np
import pytest

import oracle
from istio_amd import workloads as W
from istio_amd.bags import BagBatch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mxp(libmxp):
    import istio_amd.engine as mxp
    return mxp


@pytest.mark.parametrize("cap", ["1", "16", "1000"])
def test_error_texts_past_log_capacity(mxp, monkeypatch, cap):
    monkeypatch.setenv("MXP_ERRCAP", cap)
    rules = W.fuzz_rules(300, seed=7, depth=3)
    batch = BagBatch.from_bags(W.fuzz_bags(700, seed=8), names=list(W.DEFAULT_TEST_MANIFEST))
    eng = mxp.Engine(0)
    eng.set_vocabulary(W.DEFAULT_TEST_MANIFEST)
    eng.compile(rules)
    match, err = eng.eval_batch(batch)
    codes = mxp.bits_to_codes(match, err, len(rules))
    assert eng.error_count() > int(cap)  # the log overflowed
    ev = oracle.OracleEvaluator(W.DEFAULT_TEST_MANIFEST)
    errs = np.argwhere(codes == 2)
    rng = np.random.default_rng(1)
    errs = errs[rng.choice(len(errs), min(300, len(errs)), replace=False)]
    for q, r in errs:
        st, msg = ev.eval_predicate(rules[r], batch, int(q))
        gmsg = eng.pair_error(int(q), int(r))
        assert gmsg != "", (rules[r], int(q))
        assert gmsg == msg or (st == "panic" and gmsg in mxp.PANIC_TEXTS), (rules[r], int(q), gmsg, msg)
    # pairs that did not fail still report ""
    ok = np.argwhere(codes < 2)[:50]
    assert all(eng.pair_error(int(q), int(r)) == "" for q, r in ok)


def test_resolver_pred_error_text_past_log_capacity(mxp, monkeypatch):
    """mxp_resolve_batch's PRED_ERROR text with a one-record log equals the full-log text."""
    texts = []
    for cap in ("1", str(1 << 23)):
        monkeypatch.setenv("MXP_ERRCAP", cap)
        manifest, rules, conf, batch = W.resolver_workload(n_rules=400, n_requests=1500, seed=23)
        eng = mxp.Engine(0)
        eng.set_vocabulary(manifest)
        eng.compile(rules)
        eng.set_resolver(**conf)
        status, err_rule, sel = eng.resolve(batch, 0)
        bad = np.nonzero(status == 3)[0]
        assert len(bad) > 10
        texts.append([(int(q), int(err_rule[q]), eng.pair_error(int(q), int(err_rule[q]))) for q in bad])
    assert texts[0] == texts[1]
    assert all(t for _, _, t in texts[0])


@pytest.mark.parametrize("wl", ["fuzz", "fuzz-vt", "c1", "c4"])
def test_compact_error_output(mxp, monkeypatch, wl):
    """mxp_batch_eval_device_compact: the same match bitmap and hit counters as the bitmap form, and
    d_req_err[q] == (some error bit of request q is set)."""
    import torch
    if wl.startswith("fuzz"):
        if wl == "fuzz-vt":
            monkeypatch.setenv("MXP_DEBUG_FLAGS", "262144")
        manifest = W.DEFAULT_TEST_MANIFEST
        rules = W.fuzz_rules(500, seed=71, depth=3)
        batch = BagBatch.from_bags(W.fuzz_bags(3000 + 13, seed=72), names=list(manifest))
    elif wl == "c1":
        manifest, rules, batch = W.c1_workload(5000)
    else:
        manifest, rules, batch = W.c4_workload(n_rules=3000, n_requests=20000, seed=73)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    db = eng.upload(batch)
    Wd = (len(rules) + 31) // 32
    dm = torch.zeros((Wd, batch.n), dtype=torch.int32, device="cuda:0")
    de = torch.zeros_like(dm)
    h1 = torch.zeros(len(rules), dtype=torch.int64, device="cuda:0")
    db.eval_hits(dm.data_ptr(), de.data_ptr(), h1.data_ptr(), 0)
    dm2 = torch.full_like(dm, -1)
    flags = torch.full((batch.n,), 7, dtype=torch.uint8, device="cuda:0")
    h2 = torch.zeros_like(h1)
    db.eval_compact(dm2.data_ptr(), flags.data_ptr(), h2.data_ptr(), 0)
    torch.cuda.synchronize()
    assert torch.equal(dm, dm2) and torch.equal(h1, h2)
    want = (de != 0).any(dim=0).to(torch.uint8)
    assert torch.equal(flags, want)
    assert 0 < int(want.sum()) or wl == "c4"
    db.free()
