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
