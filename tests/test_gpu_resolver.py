"""GPU batched resolver (mxp_resolve_batch) against the resolver restatement (oracle/resolver.py):
the reference's own resolver table, then randomized namespaces / varieties / TCP flags / empty
matches / identity failures over guard-heavy rules.  Bar: identical status, first-error rule (and
its error text) and selected-rule lists, per request."""
import json
import os

import numpy as np
import pytest

import oracle
import resolver as oracle_resolver
from istio_amd import workloads as W
from istio_amd.bags import BagBatch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "resolver_cases.json")))
MANIFEST = {"destination.service": "STRING", "context.protocol": "STRING", "as": "STRING"}


@pytest.fixture(scope="module")
def mxp(libmxp):
    import istio_amd.engine as mxp
    return mxp


@pytest.mark.parametrize("case", CASES["cases"], ids=[c["desc"] for c in CASES["cases"]])
def test_reference_resolver_table_on_gpu(mxp, case):
    from test_resolver_oracle import case_inputs
    rule_ns, lengths, _ = case_inputs(case)
    match = 'as == "x"' if case.get("selectError") else ("false" if case.get("selectReject") else "true")
    eng = mxp.Engine(0)
    eng.set_vocabulary(MANIFEST)
    assert (eng.compile([match] * len(rule_ns)) == 0).all()
    n = len(rule_ns)
    eng.set_resolver(CASES["identity_attr"], CASES["default_ns"], rule_ns, [1] * n, [0] * n, [0] * n)
    batch = BagBatch.from_bags([dict(case["bag"])], names=list(MANIFEST))
    status, err_rule, sel = eng.resolve(batch, case.get("callVariety", 0))
    if "err" in case:
        if "identity" in case["err"]:
            assert status[0] == eng.RESOLVE_NO_IDENTITY
        else:
            assert status[0] == eng.RESOLVE_PRED_ERROR
            assert eng.pair_error(0, int(err_rule[0])) == "lookup failed: 'as'"
        return
    assert status[0] == eng.RESOLVE_OK
    assert sum(lengths[int(r)] for r in sel[0]) == case["nactions"]


# resolution paths: compact (default: error flags + records, device namespaces and scan), the error
# bitmap (MXP_DEBUG_FLAGS bit 28), records past a tiny log (the compact path falls back to the bitmap),
# the host packer (host namespaces), u16 rule ids (mxp_resolve_batch_ex), and the per-lane walk of
# the bitmaps instead of the tiled one (MXP_RESOLVE_TILE=0), with the error bitmap and without
MODES = {"compact": {}, "bitmap": {"MXP_DEBUG_FLAGS": "268435456"}, "errcap": {"MXP_ERRCAP": "16"},
         "hostpack": {"MXP_HOST_PACK": "1"}, "u16": {}, "lanewalk": {"MXP_RESOLVE_TILE": "0"},
         "lanewalk_bitmap": {"MXP_RESOLVE_TILE": "0", "MXP_DEBUG_FLAGS": "268435456"},
         "eager_records": {"MXP_LAZY_RECORDS": "0"}}


@pytest.mark.parametrize("seed,mode", [(21, "compact"), (22, "compact"), (21, "bitmap"), (22, "errcap"),
                                       (21, "hostpack"), (22, "u16"), (23, "lanewalk"), (23, "lanewalk_bitmap"),
                                       (23, "compact"), (23, "bitmap"), (24, "eager_records")])
def test_resolver_random_parity(mxp, monkeypatch, seed, mode):
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    manifest, rules, conf, batch = W.resolver_workload(n_rules=600, n_requests=3000, seed=seed)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    st = eng.compile(rules)
    eng.set_resolver(conf["identity_attr"], conf["default_ns"], conf["rule_ns"], conf["variety_mask"],
                     conf["is_tcp"], conf["empty_match"])
    ev = oracle.OracleEvaluator(manifest)
    codes = oracle.oracle_matrix(ev, rules, batch, threads=16)
    seen = set()
    for variety in (0, 2, 3):
        status, err_rule, sel = eng.resolve(batch, variety, ids16=mode == "u16")
        want = oracle_resolver.resolve(batch, codes, conf["rule_ns"], conf["variety_mask"], conf["is_tcp"],
                                       conf["empty_match"], conf["identity_attr"], conf["default_ns"], variety)
        for q, (ws, we, wsel) in enumerate(want):
            assert status[q] == ws, (q, variety, status[q], ws)
            seen.add(ws)
            if ws == oracle_resolver.PRED_ERROR:
                assert err_rule[q] == we, (q, variety)
                st_, msg = ev.eval_predicate(rules[we], batch, q)
                gmsg = eng.pair_error(q, int(we))
                assert gmsg == msg or (st_ == "panic" and gmsg in mxp.PANIC_TEXTS), (rules[we], gmsg, msg)
            else:
                assert list(sel[q]) == wsel, (q, variety)
    assert seen == {0, 1, 2, 3}


@pytest.mark.parametrize("extra", [{}, {"MXP_DEBUG_FLAGS": "268435456"}, {"MXP_ERRCAP": "16"}])
def test_resolver_tiled_equals_lane_walk(mxp, monkeypatch, extra):
    """The tiled walk of the default namespace (resolve.hip resolve_tile: 64-word chunks through LDS)
    over a rule set of several chunks equals the per-lane walk (MXP_RESOLVE_TILE=0), checked above
    against the oracle: status, first errors, offsets and ids, u32 and u16, for three varieties."""
    for k, v in extra.items():
        monkeypatch.setenv(k, v)
    manifest, rules, conf, batch = W.resolver_workload(n_rules=2700, n_requests=5000, seed=25)
    got = {}
    for tile in ("1", "0"):
        monkeypatch.setenv("MXP_RESOLVE_TILE", tile)
        eng = mxp.Engine(0)
        eng.set_vocabulary(manifest)
        eng.compile(rules)
        eng.set_resolver(conf["identity_attr"], conf["default_ns"], conf["rule_ns"], conf["variety_mask"],
                         conf["is_tcp"], conf["empty_match"])
        got[tile] = [[x.copy() for x in eng.resolve_arrays(batch, v, ids16=u16)] for v in (0, 2, 3)
                     for u16 in (False, True)]
        eng.close()
    for a, b in zip(got["1"], got["0"]):
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
    st, _, off, _ = got["1"][0]
    assert (st == 0).sum() > 1000 and (st == 3).sum() > 10 and int(off[-1]) > 5000


@pytest.mark.parametrize("seed", [23, 24])
def test_resolver_referenced_parity(mxp, seed):
    """mxp_resolve_refs: each Resolve's referenced attributes -- identity, context.protocol, and the
    reads of the predicates filterActions evaluates up to the first failing one -- against the
    resolver restatement's trace replayed through the oracle's FakeBag tracking; resolution results
    equal mxp_resolve_batch's."""
    from test_gpu_refs import expected_protobag
    manifest, rules, conf, batch = W.resolver_workload(n_rules=400, n_requests=1200, seed=seed)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    st = eng.compile(rules)
    keep = [i for i, s in enumerate(st) if s != 5]  # unsupported constructs have unknown reads
    if len(keep) != len(rules):
        rules = [rules[i] for i in keep]
        conf = {k: ([v[i] for i in keep] if isinstance(v, list) else v) for k, v in conf.items()}
        eng.compile(rules)
    eng.set_resolver(conf["identity_attr"], conf["default_ns"], conf["rule_ns"], conf["variety_mask"],
                     conf["is_tcp"], conf["empty_match"])
    ev = oracle.OracleEvaluator(manifest)
    codes = oracle.oracle_matrix(ev, rules, batch, threads=16)
    for variety in (0, 3):
        status, err_rule, sel, refs = eng.resolve_refs(batch, variety)
        s2, e2, sel2 = eng.resolve(batch, variety)
        assert np.array_equal(status, s2) and np.array_equal(err_rule[status == 3], e2[status == 3])
        assert all(np.array_equal(a, b) for a, b in zip(sel, sel2))
        want = oracle_resolver.resolve(batch, codes, conf["rule_ns"], conf["variety_mask"], conf["is_tcp"],
                                       conf["empty_match"], conf["identity_attr"], conf["default_ns"], variety,
                                       trace=True)
        for q, w in enumerate(want):
            exp = [x.decode("utf-8", "surrogateescape")
                   for x in oracle_resolver.resolve_referenced(ev, rules, batch, q, w[3])]
            assert mxp.fakebag_list(refs[q]) == exp, (q, variety, sorted(set(mxp.fakebag_list(refs[q])) ^ set(exp)))
            assert mxp.protobag_set(refs[q]) == expected_protobag(batch, q, exp)


def test_resolver_compact_matches_bitmap_value_classes(mxp, monkeypatch):
    """C4 routes and header rules (value-class columns; missing headers give class error records that
    the compact path expands per request): the compact Resolve equals the error-bitmap Resolve, with
    the rules spread over three namespaces and mixed varieties / TCP flags."""
    manifest, rules, batch = W.c4_workload(n_rules=1200, n_requests=20000, seed=31, cont_frac=0.2)
    manifest = dict(manifest, **{"context.protocol": "STRING"})
    # value-class rules that fail per class (no header value converts to an IP): class records;
    # placed among the default namespace's rules with variety 1 only
    bad = ['ip(request.headers["%s"]) == ip("10.0.0.1")' % h for h in ("x-user", "x-env", "x-canary", "user-agent",
                                                                     "x-region")] * 3
    rules = list(rules[:300]) + bad + list(rules[300:])
    R = len(rules)
    rng = np.random.default_rng(5)
    counts = rng.multinomial(R - 700, [0.5, 0.3, 0.2])
    counts[0] += 700
    rule_ns = ["istio-system"] * counts[0] + ["default"] * counts[1] + ["other"] * counts[2]
    vm = rng.integers(0, 8, size=R).astype(np.uint32)
    vm[300:300 + len(bad)] = 2
    tcp = (rng.random(R) < 0.1).astype(np.uint8)
    empty = (rng.random(R) < 0.02).astype(np.uint8)
    out = {}
    for mode in ("compact", "bitmap", "u16"):
        monkeypatch.setenv("MXP_DEBUG_FLAGS", MODES.get(mode, {}).get("MXP_DEBUG_FLAGS", "0"))
        eng = mxp.Engine(0)
        eng.set_vocabulary(manifest)
        assert (eng.compile(rules) == 0).all()
        eng.set_resolver("destination.service", "istio-system", rule_ns, vm, tcp, empty)
        res = []
        for variety in (0, 1, 2):
            st, er, off, sel = eng.resolve_arrays(batch, variety, ids16=mode == "u16")
            res.append((st, er, off, sel.astype(np.uint32)))
            if mode == "compact":  # every failing request's text is there
                for q in np.nonzero(st == 3)[0][:50]:
                    assert eng.pair_error(int(q), int(er[q]))
        out[mode] = res
        eng.close()
    for mode in ("bitmap", "u16"):
        for (a, b) in zip(out["compact"], out[mode]):
            for x, y in zip(a, b):
                assert np.array_equal(x, y), mode
    assert any((r[0] == 3).any() for r in out["compact"]) and any((r[0] == 0).any() for r in out["compact"])
