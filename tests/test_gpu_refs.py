"""GPU referenced attributes (mxp_eval_refs) against the reference's golden `Referenced` lists and
the oracle's FakeBag tracking (oracle_referenced), plus the ProtoBag conditions derived from the
bags.  Bar: exact set equality per request."""
import json
import os

import numpy as np
import pytest

import oracle
from istio_amd import workloads as W
from istio_amd.bags import ABSENT, STRING_MAP, BagBatch, from_tagged

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROWS = json.load(open(os.path.join(HERE, "golden", "ilt_tests.json")))


@pytest.fixture(scope="module")
def mxp(libmxp):
    import istio_amd.engine as mxp
    return mxp


def _bstr(batch, sid):
    return bytes(batch.str_blob[int(batch.str_offsets[sid]):int(batch.str_offsets[sid + 1])])


def expected_protobag(batch, q, fake):
    """ProtoBag conditions (protoBag.go:78-159) of a FakeBag list: absent -> ABSENCE, a string map
    found -> not recorded, other values -> EXACT; map keys by presence."""
    from istio_amd.engine import REF_ABSENCE, REF_EXACT
    out = set()
    for ent in fake:
        name, key = ent, None
        if ent.endswith("]") and "[" in ent:
            name, key = ent[:-1].split("[", 1)
        c = batch.names.index(name) if name in batch.names else -1
        kind = int(batch.kinds[c][q]) if c >= 0 else ABSENT
        if key is None:
            if kind == STRING_MAP:
                continue
            out.add((name, "", REF_ABSENCE if kind == ABSENT else REF_EXACT))
        else:
            m = int(batch.values[c][q])
            keys = {_bstr(batch, int(batch.map_keys[e])) for e in range(int(batch.map_offsets[m]), int(batch.map_offsets[m + 1]))}
            out.add((name, key, REF_EXACT if key.encode() in keys else REF_ABSENCE))
    return out


def test_golden_referenced_on_gpu(mxp):
    """Rows of mixer/pkg/il/testing/tests.go with a `Referenced` list, one rule per row."""
    checked = 0
    for conf in ("defaultAttrs", "exprEvalAttrs"):
        rows = [r for r in ROWS["rows"] if r.get("E") and r.get("conf", "defaultAttrs") == conf and "Referenced" in r
                and "CompileErr" not in r and "Externs" not in r]
        for r in rows:
            eng = mxp.Engine(0)
            eng.set_vocabulary(ROWS["manifests"][conf])
            assert (eng.compile([r["E"]]) == 0).all()
            batch = BagBatch.from_bags([{k: from_tagged(v) for k, v in r.get("I", {}).items()}],
                                       names=list(ROWS["manifests"][conf]))
            _, _, refs = eng.eval_refs(batch)
            assert mxp.fakebag_list(refs[0]) == r["Referenced"], r["E"]
            assert mxp.protobag_set(refs[0]) == expected_protobag(batch, 0, r["Referenced"]), r["E"]
            checked += 1
    assert checked >= 45


def _workload(name):
    if name == "c1":
        return W.c1_workload(n_bags=600)
    if name == "c2":
        return W.c2_workload(n_rules=400, n_requests=1500, seed=3)
    if name == "c4":
        return W.c4_workload(n_rules=300, n_requests=600, seed=4)
    manifest = W.DEFAULT_TEST_MANIFEST
    if name == "fuzz":
        rules = W.fuzz_rules(300, seed=5, depth=3)
    else:
        rules = W.guarded_fuzz_rules(400, seed=6)
    return manifest, rules, BagBatch.from_bags(W.fuzz_bags(500, seed=7), names=list(manifest))


@pytest.mark.parametrize("name", ["c1", "c2", "c4", "fuzz", "gfuzz"])
def test_refs_parity(mxp, name):
    """Every request's referenced set (all rules evaluated) against the oracle's FakeBag tracking:
    guard columns, composite second atoms, VM continuations, map keys; the bitmaps equal
    mxp_eval_batch's."""
    manifest, rules, batch = _workload(name)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    st = eng.compile(rules)
    rules_ok = [r for r, s in zip(rules, st) if s != 5]
    if len(rules_ok) != len(rules):  # unsupported constructs: refs are refused; test the rest
        eng.compile(rules_ok)
        rules = rules_ok
    match, err, refs = eng.eval_refs(batch)
    m2, e2 = eng.eval_batch(batch)
    assert np.array_equal(match, m2) and np.array_equal(err, e2)
    ev = oracle.OracleEvaluator(manifest)
    nonempty = 0
    for q in range(batch.n):
        want = [x.decode("utf-8", "surrogateescape") for x in oracle.oracle_referenced(ev, rules, batch, q)]
        got = mxp.fakebag_list(refs[q])
        assert got == want, (q, sorted(set(got) ^ set(want)))
        assert mxp.protobag_set(refs[q]) == expected_protobag(batch, q, want)
        nonempty += bool(want)
    assert nonempty > batch.n // 2
