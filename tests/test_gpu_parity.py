"""GPU parity: the HIP engine (libmxp, through the C-ABI) against the oracle, pair by pair.

Bar: bit-exact.  Every (request, rule) pair must agree on {false, true, error, panic} (EvalPredicate
semantics), and every error pair's message must equal the reference's text.
"""
import json
import os

import numpy as np
import pytest

import oracle
from istio_amd import workloads as W
from istio_amd.bags import BagBatch, from_tagged

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROWS = json.load(open(os.path.join(HERE, "golden", "ilt_tests.json")))


@pytest.fixture(scope="module")
def mxp(libmxp):
    import istio_amd.engine as mxp
    return mxp


def gpu_codes(engine, batch):
    """Per-pair codes from the GPU bitmaps, with panics told apart through the error log."""
    match, err = engine.eval_batch(batch)
    codes = __import__("istio_amd.engine", fromlist=["x"]).bits_to_codes(match, err, len(engine.rules))
    return codes


def compare(engine, ev, rules, batch, sample_msgs=400, seed=0):
    from istio_amd.engine import PANIC_TEXTS
    got = gpu_codes(engine, batch)
    want = oracle.oracle_matrix(ev, rules, batch, threads=16)
    want_err = np.where(want >= 2, 2, want)  # bitmaps carry error|panic in one bit
    bad = np.argwhere(got != want_err)
    assert bad.size == 0, "first mismatches (req, rule, got, want): %s; rules: %s" % (
        [(int(q), int(r), int(got[q, r]), int(want_err[q, r])) for q, r in bad[:5]], [rules[j] for _, j in bad[:3]])
    # error texts (and error-vs-panic class) for a sample of error pairs
    errs = np.argwhere(want >= 2)
    rng = np.random.default_rng(seed)
    if len(errs) > sample_msgs:
        errs = errs[rng.choice(len(errs), sample_msgs, replace=False)]
    for q, r in errs:
        st, msg = ev.eval_predicate(rules[r], batch, int(q))
        gmsg = engine.pair_error(int(q), int(r))
        assert gmsg == msg or (st == "panic" and gmsg in PANIC_TEXTS), (rules[r], int(q), gmsg, msg)
        assert (gmsg in PANIC_TEXTS) == (st == "panic"), (rules[r], gmsg, st)
    return got, want


def test_golden_double_session_on_gpu(mxp):
    """compiler_test.go:87-136 (TestCompiler_DoubleExpressionSession): every golden expression
    compiled twice into one rule set; on the GPU both copies give the same code, value and error
    text on their row's bag as the single compile."""
    for conf in ("defaultAttrs", "exprEvalAttrs"):
        rows = [r for r in ROWS["rows"] if r.get("E") and r.get("conf", "defaultAttrs") == conf
                and "CompileErr" not in r and "Externs" not in r]
        batch = BagBatch.from_bags([{k: from_tagged(v) for k, v in r.get("I", {}).items()} for r in rows])
        single = mxp.Engine(0)
        single.set_vocabulary(ROWS["manifests"][conf])
        single.compile([r["E"] for r in rows])
        sv, sc = single.eval_values(batch)
        eng = mxp.Engine(0)
        eng.set_vocabulary(ROWS["manifests"][conf])
        st = eng.compile([r["E"] for r in rows for _ in (0, 1)])
        assert (st == 0).all()
        vals, codes = eng.eval_values(batch)
        pm, pe = eng.eval_batch(batch)
        pcodes = mxp.bits_to_codes(pm, pe, 2 * len(rows))
        for i, r in enumerate(rows):
            a, b = 2 * i, 2 * i + 1
            assert codes[i, a] == codes[i, b] == sc[i, i], r["E"]
            assert pcodes[i, a] == pcodes[i, b], r["E"]
            if codes[i, a] >= 2:
                assert eng.pair_error(i, a) == eng.pair_error(i, b) == single.pair_error(i, i), r["E"]
            else:
                assert eng.value_text(a, vals[i, a]) == eng.value_text(b, vals[i, b]) == \
                    single.value_text(i, sv[i, i]), r["E"]


def test_golden_table_on_gpu(mxp):
    """Every golden row (mixer/pkg/il/testing/tests.go) evaluated by the GPU engine."""
    from test_oracle_golden import same_value
    for conf in ("defaultAttrs", "exprEvalAttrs"):
        rows = [r for r in ROWS["rows"] if r.get("E") and r.get("conf", "defaultAttrs") == conf
                and "CompileErr" not in r and "Externs" not in r]
        eng = mxp.Engine(0)
        eng.set_vocabulary(ROWS["manifests"][conf])
        st = eng.compile([r["E"] for r in rows])
        assert (st == 0).all(), [rows[i]["E"] for i in np.where(st != 0)[0]]
        batch = BagBatch.from_bags([{k: from_tagged(v) for k, v in r.get("I", {}).items()} for r in rows])
        vals, codes = eng.eval_values(batch)
        # predicate mode (guards + VM) must agree with Eval mode on every bool row
        pm, pe = eng.eval_batch(batch)
        pcodes = mxp.bits_to_codes(pm, pe, len(rows))
        for i, r in enumerate(rows):
            if r.get("Type") == "BOOL" or "Err" in r:
                assert pcodes[i, i] == min(int(codes[i, i]), 2), r["E"]
        for i, r in enumerate(rows):
            c = int(codes[i, i])
            if "Err" in r:
                assert c in (2, 3), r["E"]
                assert eng.pair_error(i, i).startswith(r["Err"]), (r["E"], eng.pair_error(i, i))
                continue
            assert c in (0, 1), (r["E"], eng.pair_error(i, i))
            want = from_tagged(r["R"])
            got = mxp.decode_value(eng, i, int(vals[i, i]))
            if isinstance(want, (bool, bytes)) or type(want).__name__ in ("GoInt64", "GoFloat64", "GoDuration"):
                assert same_value(want, got), (r["E"], want, got)
            elif isinstance(want, str):
                assert got == want, (r["E"], want, got)
            else:  # time.Time results (mxp_value_decode: Unix seconds + nanoseconds) and string maps
                assert got == want, (r["E"], want, got)


def test_c1_bookinfo_parity(mxp):
    manifest, rules, batch = W.c1_workload(10000)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    ev = oracle.OracleEvaluator(manifest)
    got, want = compare(eng, ev, rules, batch)
    assert (want == 1).any() and (want == 2).any()


def test_c2_parity_config_size(mxp):
    """BASELINE configs[1]: 1k rules x 64k requests, full pair matrix against the oracle."""
    manifest, rules, batch = W.c2_workload(n_rules=1000, n_requests=65536)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    ev = oracle.OracleEvaluator(manifest)
    got, want = compare(eng, ev, rules, batch)
    assert (want == 1).sum() > 0 and (want == 2).sum() > 0


def test_c4_routes_parity(mxp):
    """BASELINE configs[3] family (Pilot-style routes: prefixes, regexes on the path and on headers),
    300 rules x 2000 requests against the oracle (Go regexp restatement for `matches`)."""
    manifest, rules, batch = W.c4_workload(n_rules=300, n_requests=2000, seed=4)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    assert eng.ruleset_info()["indexed"] > 0.7 * len(rules)  # prefix index: startsWith + anchored regexps
    ev = oracle.OracleEvaluator(manifest)
    got, want = compare(eng, ev, rules, batch)
    assert (want == 1).sum() > 500


@pytest.mark.parametrize("seed", [7, 17])
def test_fuzz_parity(mxp, seed):
    """Random well- and ill-typed rules over random bags with missing / wrongly typed values, plus
    the rules at the reference VM's limits (workloads.hard_fuzz_rules: long chains to heap slot 63,
    index panics after an ip() return, `|` chains past the 64-word stack, right-nested comparisons
    for the deep kernels, run-time regexp patterns).  Every rule compiles: no MXP_RULE_UNSUPPORTED."""
    rules = W.fuzz_rules(600, seed=seed, depth=3) + W.hard_fuzz_rules(300, seed=seed + 2)
    bags = W.fuzz_bags(400, seed=seed + 1)
    bags += W.fuzz_bags(200, seed=seed + 3, p_missing=0.03, p_wrong=0.01)
    batch = BagBatch.from_bags(bags, names=list(W.DEFAULT_TEST_MANIFEST))
    eng = mxp.Engine(0)
    eng.set_vocabulary(W.DEFAULT_TEST_MANIFEST)
    st = eng.compile(rules)
    assert (st != 5).all(), [(rules[i][:80], eng.rule_error(i)) for i in np.where(st == 5)[0][:3]]
    ev = oracle.OracleEvaluator(W.DEFAULT_TEST_MANIFEST)
    compare(eng, ev, rules, batch)


@pytest.mark.parametrize("knobs", [{}, {"MXP_DEBUG_FLAGS": "8"}, {"MXP_HOST_PACK": "1"}])
def test_reference_limits_parity(mxp, knobs, monkeypatch):
    """Rules that reach the reference VM's limits evaluate as the reference does instead of being
    refused: "heap overflow" at slot 63 (interpreterRun.go:171-172), Go's index panic when an ip()
    return took slot 63 (extern.go:232-237), "stack overflow" past 64 words, deep nesting in the
    64-register kernels, and `matches` patterns computed at run time (externs.go:118-120).  Every
    error pair's text is compared (compare(sample_msgs=10**6))."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    whitelist = " || ".join('as == "x%d"' % i for i in range(70))
    rules = [whitelist, "(%s) && bs == \"abc\"" % whitelist, '(ar["a"] | "^x").matches(bs)',
             '(ar["a"] | as).matches(bs)', '(ar[as] | "^a").matches(bs)', '(sm["b"] | br["a"] | "(x").matches(as)',
             " || ".join('as == "x%d"' % i for i in range(62)) + ' || ip(as) == ip("1.2.3.4") || bs == "abc"',
             " | ".join("(ai == %d)" % (i % 3) for i in range(70)), " | ".join('(as == "a%d")' % i for i in range(70)),
             "ab == (" * 20 + "bb" + ")" * 20]
    rules += W.hard_fuzz_rules(400, seed=5)
    bags = W.fuzz_bags(600, seed=6, p_missing=0.03, p_wrong=0.01) + W.fuzz_bags(200, seed=9)
    for i, b in enumerate(bags[:100]):  # whitelist hits at every position
        b["as"] = "x%d" % (i % 72)
    batch = BagBatch.from_bags(bags, names=list(W.DEFAULT_TEST_MANIFEST))
    eng = mxp.Engine(0)
    eng.set_vocabulary(W.DEFAULT_TEST_MANIFEST)
    st = eng.compile(rules)
    assert (st == 0).all(), [(rules[i][:80], eng.rule_error(i)) for i in np.where(st != 0)[0][:3]]
    ev = oracle.OracleEvaluator(W.DEFAULT_TEST_MANIFEST)
    got, want = compare(eng, ev, rules, batch, sample_msgs=1500)
    texts = {ev.eval_predicate(rules[r], batch, int(q))[1] for q, r in np.argwhere(want >= 2)[:20000:7]}
    assert {"heap overflow", "stack overflow", "runtime error: index out of range"} <= texts, texts
    assert (want[:, 0] == 1).sum() >= 60 and (want[:, 0] == 2).sum() > 100  # whitelist: hits, then heap overflow
    # Eval mode runs whole programs (no guards, no index) through the same kernels
    vals, codes = eng.eval_values(batch)
    pc = np.where(want >= 2, 2, want)
    boolean = np.array([eng.rule_types(i)[1] == 5 for i in range(len(rules))])
    assert np.array_equal(np.minimum(codes[:, boolean], 2), pc[:, boolean])


@pytest.mark.parametrize("knobs", [{}, {"MXP_DEBUG_FLAGS": "8"}, {"MXP_GPW": "1"}, {"MXP_DEBUG_FLAGS": "65536"}])
def test_guarded_fuzz_parity(mxp, knobs, monkeypatch):
    """Guard-led rules (mixed columns / want classes / negations / modes per group, shared and
    singleton continuation templates, indexed and in-wave continuations) under each routing:
    default (guard index on), guard index off (MXP_DEBUG_FLAGS=8: every continuation in-wave), one
    group per wave, the one-request-per-lane lean kernel (MXP_DEBUG_FLAGS=65536)."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    rules = W.guarded_fuzz_rules(2000, seed=11)
    # 4096 + 37: a partial last workgroup (the lean kernels' 128-request tiles load ABSENT past the end)
    bags = W.fuzz_bags(4096 + 37, seed=12)
    batch = BagBatch.from_bags(bags, names=list(W.DEFAULT_TEST_MANIFEST))
    eng = mxp.Engine(0)
    eng.set_vocabulary(W.DEFAULT_TEST_MANIFEST)
    eng.compile(rules)
    info = eng.ruleset_info()
    assert info["templated"] > 500 and info["templates"] > 50
    assert info["indexed"] > 300 or knobs.get("MXP_DEBUG_FLAGS") == "8"
    ev = oracle.OracleEvaluator(W.DEFAULT_TEST_MANIFEST)
    got, want = compare(eng, ev, rules, batch, sample_msgs=200)
    assert (want == 1).sum() > 1000 and (want >= 2).sum() > 1000


def test_device_resident_batch_and_hits(mxp):
    """mxp_batch_upload + mxp_batch_eval_device + mxp_hits_device agree with the host path."""
    import torch
    manifest, rules, batch = W.c2_workload(n_rules=300, n_requests=20000)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    match_h, err_h = eng.eval_batch(batch)
    db = eng.upload(batch)
    W_ = (len(rules) + 31) // 32
    dm = torch.zeros((W_, batch.n), dtype=torch.int32, device="cuda:0")
    de = torch.zeros_like(dm)
    hits = torch.zeros(len(rules), dtype=torch.int64, device="cuda:0")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    db.eval(dm.data_ptr(), de.data_ptr(), s.cuda_stream)
    rc = eng.lib.mxp_hits_device(eng.h, dm.data_ptr(), batch.n, s.cuda_stream, hits.data_ptr())
    assert rc == 0
    torch.cuda.synchronize()
    assert np.array_equal(dm.cpu().numpy().view(np.uint32), match_h)
    assert np.array_equal(de.cpu().numpy().view(np.uint32), err_h)
    codes = mxp.bits_to_codes(match_h, err_h, len(rules))
    assert np.array_equal(hits.cpu().numpy(), (codes == 1).sum(axis=0))


@pytest.mark.parametrize("n", [1, 3, 64, 1001, 4100, 1 << 20, (1 << 20) + 7])
def test_hits_counts_random_bitmaps(mxp, n):
    """mxp_hits_device's bit-sliced counting against numpy on random bitmaps of every density: the
    16-byte path (n % 4 == 0), the scalar path (ragged n) and partial last steps."""
    import torch
    rng = np.random.default_rng(n)
    R = 70  # three words, the last one partial
    Wd = (R + 31) // 32
    dens = rng.choice([0.0, 0.01, 0.5, 0.99, 1.0], size=(Wd, 1, 32))
    bits = rng.random((Wd, n, 32)) < dens
    words = np.ascontiguousarray(np.packbits(bits, axis=2, bitorder="little")).view("<u4").reshape(Wd, n)
    eng = mxp.Engine(0)
    eng.set_vocabulary({"a": "STRING"})
    eng.compile(['a == "x"'] * R)
    dm = torch.from_numpy(words.view(np.int32)).to("cuda:0")
    hits = torch.full((R,), 5, dtype=torch.int64, device="cuda:0")
    rc = eng.lib.mxp_hits_device(eng.h, dm.data_ptr(), n, torch.cuda.current_stream().cuda_stream, hits.data_ptr())
    assert rc == 0
    torch.cuda.synchronize()
    want = bits.sum(axis=1).reshape(-1)[:R] + 5
    assert np.array_equal(hits.cpu().numpy(), want)


def composite_rules(n, seed=31):
    """`A == K1 && B.startsWith(K2) [&& tail]` rules (composite index), mixed with look-alikes the
    index must not take: a tail that re-reads B, `||` forms, negated atoms, VCOL columns."""
    rng = np.random.default_rng(seed)
    vals = W._STR_VALS
    pre = ["", "a", "ab", "abc", "abcd", "st", "1.2", "10.0", "2015-01-02T", "*"]
    tails = ["", ' && ai == %d' % 2, ' && aip != ip("1.2.3.4")', ' && bs == "abc"', ' && ab', ' || ai == 1',
             ' && "^a".matches(bs)', ' && ar["a"] == "abc"']
    out = []
    for _ in range(n):
        a = rng.choice(["as", "bs", 'ar["%s"]' % rng.choice(W._KEYS)])
        b = rng.choice(["bs", "as", "bs"])
        out.append('%s == "%s" && %s.startsWith("%s")%s' % (a, rng.choice(vals), b, rng.choice(pre),
                                                           rng.choice(tails)))
    return out


def test_composite_index_parity(mxp):
    """Composite guard index (A == K1 && B.startsWith(K2) && ...): B missing, of the wrong type,
    shorter than K2, K2 empty, several K2 lengths per K1, direct and templated forms."""
    rules = composite_rules(1500)
    bags = W.fuzz_bags(6000, seed=33, p_missing=0.2, p_wrong=0.05)
    batch = BagBatch.from_bags(bags, names=list(W.DEFAULT_TEST_MANIFEST))
    eng = mxp.Engine(0)
    eng.set_vocabulary(W.DEFAULT_TEST_MANIFEST)
    st = eng.compile(rules)
    info = eng.ruleset_info()
    assert info["composite"] > 400, info
    ev = oracle.OracleEvaluator(W.DEFAULT_TEST_MANIFEST)
    got, want = compare(eng, ev, rules, batch, sample_msgs=300)
    assert (want == 1).sum() > 2000 and (want >= 2).sum() > 2000


@pytest.mark.parametrize("n", [1, 5, 1001, 4099])
def test_c2_ragged_batches(mxp, n):
    """Uniform indexed groups (mxp_fill_kernel) and the pair queue at batch sizes that are not a
    multiple of the 4-request lane width or of a wavefront; error texts from the log."""
    manifest, rules, batch = W.c2_workload(n_rules=333, n_requests=n, seed=7)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    ev = oracle.OracleEvaluator(manifest)
    compare(eng, ev, rules, batch, sample_msgs=100)


@pytest.mark.parametrize("knobs", [{"MXP_FILL_SPAN": "1", "MXP_FILL_CHUNK": "32"}, {"MXP_FILL_SPAN": "2"},
                                   {"MXP_FILL_SPAN": "8", "MXP_FILL_CHUNK": "5"},
                                   {"MXP_FILL_SPAN": "3", "MXP_FILL_CHUNK": "1000"}])
@pytest.mark.parametrize("n", [5, 4099, 20000])
def test_fill_layout_knobs_parity(mxp, knobs, n, monkeypatch):
    """mxp_fill_kernel's store layout knobs (MXP_FILL_SPAN: 256-request spans per wave, including
    spans past the batch end; MXP_FILL_CHUNK: groups per chunk) leave every word unchanged: oracle
    parity on ragged batches, and the pipelined device path equal to the unpipelined one."""
    import torch
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    manifest, rules, batch = W.c2_workload(n_rules=333, n_requests=n, seed=7)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    compare(eng, oracle.OracleEvaluator(manifest), rules, batch, sample_msgs=100)
    if n < 4096:
        return
    db = eng.upload(batch)
    Wd = (len(rules) + 31) // 32
    outs = []
    s = torch.cuda.current_stream().cuda_stream
    for pipe in ((2048, 4), (1 << 30, 1)):
        eng.set_pipeline(*pipe)
        dm = torch.full((Wd, batch.n), -1, dtype=torch.int32, device="cuda:0")
        de = torch.full_like(dm, -1)
        db.eval(dm.data_ptr(), de.data_ptr(), s)
        torch.cuda.synchronize()
        outs.append((dm.cpu().numpy(), de.cpu().numpy()))
    for a, b in zip(*outs):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("family", ["c2", "fuzz", "c4"])
@pytest.mark.parametrize("flags,sync", [("0", True), ("0", False), ("524288", True), ("786432", True),
                                        ("1048576", False)])  # auto; fused forced; + value classes; streaming
def test_fused_hit_counters(mxp, family, flags, sync, monkeypatch):
    """mxp_batch_eval_device_hits: counters accumulated by the evaluation kernels (fill / guard / VM
    kernels by ballot, index kernel per newly set bit) -- or, after an evaluation dense in true pairs
    (C4), by the streaming hits kernel; value-class rules per class (class size x class word) -- equal
    the true pairs of the bitmaps over three evaluations, and the bitmaps equal the plain device
    evaluation's.  The choice is made on the device from the previous evaluation (mxp_hits_gate_kernel),
    so evaluations queued back to back without a host synchronisation (sync False) count alike."""
    import torch
    monkeypatch.setenv("MXP_DEBUG_FLAGS", flags)
    if family == "c2":
        manifest, rules, batch = W.c2_workload(n_rules=700, n_requests=30000)
    elif family == "c4":
        manifest, rules, batch = W.c4_workload(n_rules=1500, n_requests=8000)
    else:
        manifest = W.DEFAULT_TEST_MANIFEST
        rules = W.guarded_fuzz_rules(1500, seed=41)
        batch = BagBatch.from_bags(W.fuzz_bags(5000, seed=42), names=list(manifest))
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    db = eng.upload(batch)
    Wd = (len(rules) + 31) // 32
    dm = torch.zeros((Wd, batch.n), dtype=torch.int32, device="cuda:0")
    de = torch.zeros_like(dm)
    dm2, de2 = torch.zeros_like(dm), torch.zeros_like(dm)
    hits = torch.full((len(rules),), 3, dtype=torch.int64, device="cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        db.eval_hits(dm.data_ptr(), de.data_ptr(), hits.data_ptr(), s)
        if sync:
            torch.cuda.synchronize()
    db.eval(dm2.data_ptr(), de2.data_ptr(), s)
    torch.cuda.synchronize()
    m = dm.cpu().numpy().view(np.uint32)
    assert np.array_equal(m, dm2.cpu().numpy().view(np.uint32))
    assert np.array_equal(de.cpu().numpy(), de2.cpu().numpy())
    codes = mxp.bits_to_codes(m, de.cpu().numpy().view(np.uint32), len(rules))
    want = 3 * (codes == 1).sum(axis=0) + 3
    assert want.sum() > 3 * len(rules)
    assert np.array_equal(hits.cpu().numpy(), want)


@pytest.mark.parametrize("knobs", [{}, {"MXP_DEBUG_FLAGS": "64"}])
def test_duplicate_rules_parity(mxp, knobs, monkeypatch):
    """Indexed rules with identical programs are evaluated once and fanned out (aliases): results,
    error bits and error records of every duplicate match the oracle; MXP_DEBUG_FLAGS=64 turns the
    dedupe off."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(61)
    base = composite_rules(200, seed=62) + W.guarded_fuzz_rules(300, seed=63)
    base += ['"^a[bc]?$".matches(bs)', '"^ab".matches(as)', 'as.startsWith("ab")', '"^a".matches(ar["a"])']
    rules = [base[i] for i in rng.integers(0, len(base), size=1500)]
    bags = W.fuzz_bags(3000, seed=64, p_missing=0.2, p_wrong=0.05)
    batch = BagBatch.from_bags(bags, names=list(W.DEFAULT_TEST_MANIFEST))
    eng = mxp.Engine(0)
    eng.set_vocabulary(W.DEFAULT_TEST_MANIFEST)
    eng.compile(rules)
    info = eng.ruleset_info()
    assert info["aliases"] > 300 or knobs, info
    ev = oracle.OracleEvaluator(W.DEFAULT_TEST_MANIFEST)
    got, want = compare(eng, ev, rules, batch, sample_msgs=400)
    assert (want == 1).sum() > 1000 and (want >= 2).sum() > 1000


@pytest.mark.parametrize("family,n,min_req,chunks", [("c2", 65536, 8192, 8), ("c2", 5000, 500, 8),
                                                     ("c4", 8000, 2048, 3), ("fuzz", 5000, 1024, 4)])
def test_pipelined_chunks_parity(mxp, family, n, min_req, chunks):
    """mxp_set_pipeline: request chunks whose guard-index pass runs on the side stream, overlapped with
    the next chunk's fill / guard / VM kernels.  Host path against the oracle, the device path (with
    fused hit counters) against the unpipelined evaluation, ragged chunk ends included."""
    import torch
    if family == "c2":
        manifest, rules, batch = W.c2_workload(n_rules=700, n_requests=n, seed=9)
    elif family == "c4":
        manifest, rules, batch = W.c4_workload(n_rules=1500, n_requests=n)
    else:
        manifest = W.DEFAULT_TEST_MANIFEST
        rules = W.guarded_fuzz_rules(1500, seed=43)
        batch = BagBatch.from_bags(W.fuzz_bags(n, seed=44), names=list(manifest))
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    eng.set_pipeline(min_req, chunks)
    if family != "fuzz":
        compare(eng, oracle.OracleEvaluator(manifest), rules, batch, sample_msgs=100)
    db = eng.upload(batch)
    Wd = (len(rules) + 31) // 32
    outs = []
    s = torch.cuda.current_stream().cuda_stream
    for pipe in ((min_req, chunks), (1 << 30, 1)):
        eng.set_pipeline(*pipe)
        dm = torch.full((Wd, batch.n), -1, dtype=torch.int32, device="cuda:0")
        de = torch.full_like(dm, -1)
        hits = torch.zeros(len(rules), dtype=torch.int64, device="cuda:0")
        db.eval_hits(dm.data_ptr(), de.data_ptr(), hits.data_ptr(), s)
        torch.cuda.synchronize()
        outs.append((dm.cpu().numpy(), de.cpu().numpy(), hits.cpu().numpy()))
    for a, b in zip(*outs):
        assert np.array_equal(a, b)
    codes = mxp.bits_to_codes(outs[0][0].view(np.uint32), outs[0][1].view(np.uint32), len(rules))
    assert np.array_equal(outs[0][2], (codes == 1).sum(axis=0))


@pytest.mark.parametrize("family", ["c1", "c2"])
def test_wire_path_parity(mxp, family):
    """Bags sent as CompressedAttributes and decoded by the engine (mxp_wire_decode, names = the rule
    set's) evaluate bit-identically to the same bags given as a columnar batch."""
    from istio_amd import wire
    if family == "c1":
        manifest, rules, batch = W.c1_workload(n_bags=3000)
    else:
        manifest, rules, batch = W.c2_workload(n_rules=500, n_requests=8000, seed=11)
    bags = [{n: v for n in batch.names for v, f in [batch.get(q, n)] if f and type(v).__name__ != "GoOther"}
            for q in range(batch.n)]
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    dec = wire.decode(eng, wire.from_bags(bags, sorted(manifest)[::3]))
    m1, e1 = eng.eval_batch(dec)
    m2, e2 = eng.eval_batch(BagBatch.from_bags(bags, names=list(manifest)))
    assert np.array_equal(m1, m2) and np.array_equal(e1, e2)
    assert m1.any()


@pytest.mark.parametrize("knobs", [{}, {"MXP_DEBUG_FLAGS": "256"}])
def test_dense_alias_injection_parity(mxp, knobs, monkeypatch):
    """Indexed rules with many duplicates ("dense" canonical rules): their true pairs are injected
    once per bitmap word at the end of the index kernel (MXP_DEBUG_FLAGS=256: per-alias atomics
    instead).  Results, error bits and fused hit counters against the oracle."""
    import torch
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    manifest, rules0, batch = W.c4_workload(n_rules=400, n_requests=6000, seed=12)
    rng = np.random.default_rng(5)
    hot = ['"^v(1|%d)[0-9]?$".matches(request.headers["x-user"])' % d for d in range(2, 9)] + \
          ['request.path.startsWith("/w1")', 'request.headers["x-env"] == "v3" && request.path.startsWith("/w2")',
           '"^/w3[0-9a-z/]*".matches(request.path)']
    rules = list(rules0) + [hot[int(i)] for i in rng.integers(0, len(hot), size=900)]
    rng.shuffle(rules)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    info = eng.ruleset_info()
    # startsWith alone and the prefix-decided `^/w3[...]*` (a direct prefix posting on "/w3") are not dense
    assert info["dense"] == (0 if knobs else len(hot) - 2)
    got, want = compare(eng, oracle.OracleEvaluator(manifest), rules, batch, sample_msgs=100)
    assert (want == 1).sum() > 10 * batch.n
    db = eng.upload(batch)
    Wd = (len(rules) + 31) // 32
    dm = torch.zeros((Wd, batch.n), dtype=torch.int32, device="cuda:0")
    de = torch.zeros_like(dm)
    hits = torch.zeros(len(rules), dtype=torch.int64, device="cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(2):  # the first evaluation counts in the kernels, the second (dense) by streaming
        db.eval_hits(dm.data_ptr(), de.data_ptr(), hits.data_ptr(), s)
    torch.cuda.synchronize()
    assert np.array_equal(hits.cpu().numpy(), 2 * (want == 1).sum(axis=0))


def test_empty_batches_and_rule_sets(mxp):
    """Edge sizes: an empty batch, an empty rule set, one request with every attribute absent --
    through the host, device, refs, resolver-free and wire entry points."""
    import torch
    from istio_amd import wire
    manifest, rules, batch = W.c2_workload(n_rules=64, n_requests=10, seed=3)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    empty = BagBatch.from_bags([], names=list(manifest))
    m, e = eng.eval_batch(empty)
    assert m.size == 0 and e.size == 0
    _, _, refs = eng.eval_refs(empty)
    assert refs == []
    db = eng.upload(empty)
    assert db.n == 0
    bare = BagBatch.from_bags([{}], names=list(manifest))
    m, e = eng.eval_batch(bare)
    codes = mxp.bits_to_codes(m, e, len(rules))
    ev = oracle.OracleEvaluator(manifest)
    want = oracle.oracle_matrix(ev, rules, bare, threads=1)
    assert np.array_equal(codes, np.where(want >= 2, 2, want))
    dec = wire.decode(eng, wire.WireBatch([], ["destination.service"]))
    assert dec.n == 0 and eng.eval_batch(dec)[0].size == 0
    none = mxp.Engine(0)
    none.set_vocabulary(manifest)
    none.compile([])
    m, e = none.eval_batch(batch)
    assert m.size == 0 and e.size == 0


UTF8_PATTERNS = ["^/api/v[0-9]+/é", "日本", "^.{3}$", "[à-ÿ]+x", "^[^a-z]*$", "😀$", "^(a|é|日)+$", ".", "^$",
                 "é.*日.*😀", "[\\x{4e00}-\\x{9fff}]{2}", "^/[a-z]+/[^/]+$", "a.b", "^[a-zé/0-9]{8,}$", "ÿ{2}|zz",
                 # Unicode classes and non-ASCII folding (parity unpinned: see test_regex_oracle.UNICODE_KAT)
                 "\\p{Han}{2}", "(?i)éΣ", "^\\pL{3}", "\\P{L}$", "(?i)[à-ö]x", "[\\p{Greek}\\p{Nd}]{2}", "(?i)\\W\\W",
                 "^\\p{Ll}+$", "\\p{So}"]


@pytest.mark.parametrize("seed", [3, 4])
def test_regex_utf8_subjects_parity(mxp, seed):
    """`matches` over subjects that mix ASCII with 2-, 3- and 4-byte UTF-8 runes, of lengths that
    cross the DFA walker's 8-byte windows at every offset: constant patterns (rule-set DFAs) and a
    pattern read from an attribute (per-batch DFAs), against the oracle's Go regexp restatement."""
    rng = np.random.default_rng(seed)
    alphabet = ["a", "b", "z", "x", "/", "0", "9", "A", "-", "é", "ÿ", "à", "日", "本", "😀", "Σ", "ς", "É", "K", "ſ"]
    weights = np.array([6, 3, 2, 2, 4, 2, 2, 1, 1, 2, 2, 1, 2, 1, 1, 1, 1, 1, 1, 1], dtype=float)
    subjects = []
    for _ in range(3000):
        L = int(rng.integers(0, 41))
        subjects.append("".join(rng.choice(alphabet, size=L, p=weights / weights.sum())))
    subjects[:4] = ["", "/api/v12/é", "日本語", "aéa"]
    manifest = {"request.path": "STRING", "x": "STRING"}
    bags = [{"request.path": s, "x": UTF8_PATTERNS[i % len(UTF8_PATTERNS)]} for i, s in enumerate(subjects)]
    batch = BagBatch.from_bags(bags, names=list(manifest))
    rules = ['"%s".matches(request.path)' % p.replace("\\", "\\\\") for p in UTF8_PATTERNS] + \
            ["x.matches(request.path)", '"^/api".matches(request.path) && "é$".matches(request.path)']
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all(), [eng.rule_error(i) for i in range(len(rules))]
    got, want = compare(eng, oracle.OracleEvaluator(manifest), rules, batch, sample_msgs=50)
    assert (want == 1).sum() > 2000 and (want == 0).sum() > 2000


def test_extern_kats_on_gpu(mxp):
    """mixer/pkg/il/runtime/externs_test.go:24-129 (tests/golden/externs_kat.json) through the GPU
    engine: the externs as predicates over attributes, pair by pair against the oracle, and the KATs'
    expected outcomes themselves."""
    from test_oracle_golden import EXTERNS, extern_bag
    manifest = {"s1": "STRING", "s2": "STRING"}
    rules = ["ip(s1) == ip(s2)", "timestamp(s1) == timestamp(s2)", "match(s1, s2)", "s1.matches(s2)"]
    batch = BagBatch.from_bags([extern_bag(c) for c in EXTERNS], names=list(manifest))
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    got, _ = compare(eng, oracle.OracleEvaluator(manifest), rules, batch)
    col = {"ip": 0, "ip_equal": 0, "timestamp": 1, "timestamp_equal": 1, "match": 2, "matches": 3}
    for q, c in enumerate(EXTERNS):
        code = int(got[q, col[c["fn"]]])
        if c.get("err"):
            assert code == 2, c
        elif isinstance(c.get("want"), bool):
            assert code == int(c["want"]), c
        else:  # ip(x) == ip(x), timestamp(x) == timestamp(x) of a valid x
            assert code == 1, c


@pytest.mark.parametrize("knobs", [{}, {"MXP_DTP": "0"}, {"MXP_DEBUG_FLAGS": "8"}])
def test_deep_continuation_guard_parity(mxp, knobs, monkeypatch):
    """Guard-led rules whose constant-free continuation needs more than MXP_VM_MAXREG registers
    (they must stay out of the guard index and the fill groups, and run in the deep
    kernels), mixed with shallow indexed rules in the same groups, deferred pairs on and off."""
    from test_product_compile import deep_continuation_rules
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    rules = deep_continuation_rules(64) + ['as == "x%d" && bs == "b%d"' % (i % 40, i % 3) for i in range(100)]
    bags = W.fuzz_bags(1500, seed=31, p_missing=0.02, p_wrong=0.01)
    rng = np.random.default_rng(32)
    for b in bags:
        if rng.random() < 0.6:
            b["as"] = "x%d" % rng.integers(0, 70)
            b["bs"] = "b%d" % rng.integers(0, 3)
    batch = BagBatch.from_bags(bags, names=list(W.DEFAULT_TEST_MANIFEST))
    eng = mxp.Engine(0)
    eng.set_vocabulary(W.DEFAULT_TEST_MANIFEST)
    assert (eng.compile(rules) == 0).all()
    ev = oracle.OracleEvaluator(W.DEFAULT_TEST_MANIFEST)
    got, want = compare(eng, ev, rules, batch)
    assert (want[:, :64] == 1).sum() > 100 and (want[:, 72:] == 1).sum() > 100


@pytest.mark.parametrize("flags", ["0", "67108864", "8"])
def test_literal_key_regexp_rules(mxp, monkeypatch, flags):
    """Prefix-guarded regexp rules whose DFA after the literal prefix is a few literal keys become
    direct postings of the prefix index -- prefix keys (any continuation matches) and exact keys (the
    subject ends there) -- with no VM pass (regex.cpp dfa_literal_keys); 67108864 keeps the DFA
    templates, 8 turns the index off.  `.*$` tails (the rest of the subject holds no newline) are
    tail keys.  Subjects around every boundary: the prefix alone, one byte more or less, the
    continuation bytes, newlines before / at / after the key, non-ASCII and invalid UTF-8 after the
    prefix."""
    monkeypatch.setenv("MXP_DEBUG_FLAGS", flags)
    pats = ["^/p(/.*)?$", "^/p[0-9a-z/]*", "^/q$", "^/q(a|bc)$", "^/r[0-9]?$", "^/s(/x|/y.*)", "^/t.{0,2}$",
            "^/u(é|e)$", "^/v\\b", "^/w(?:x|$)", "^/p/", "^/pa(b|$)", "^/n.*$", "^/k(x.*|y)$", "^/j[a-z]*.*$",
            "^/g\\n.*$", "^/i.+$", "^/h(?s:.*)$", "^/f(/[a-z]*)?.*$"]
    rules = ['"%s".matches(request.path)' % p.replace("\\", "\\\\") for p in pats]
    rules += ['request.path.startsWith("/p")', 'request.path == "/q"']
    tails = ["", "/", "/x", "/y", "/yy", "a", "b", "bc", "bcd", "0", "9", "09", "x", "é", "e", "\udcff", "\udcc3",
             "/é", " ", "-", "ab", "abc", "\n", "/\n", "/a\nb", "\nx", "x\n", "y\n", "/\udcff", "\n\n"]
    rng = np.random.default_rng(71)
    heads = ["/p", "/q", "/r", "/s", "/t", "/u", "/v", "/w", "/pa", "/", "", "/P", "/n", "/k", "/j", "/g", "/i",
             "/h", "/f", "\n/p"]
    paths = [h + t for h in heads for t in tails]
    bags = [{"request.path": p} for p in paths] + [{}] + [{"request.path": 7}]
    bags += [{"request.path": heads[int(rng.integers(0, len(heads)))] + tails[int(rng.integers(0, len(tails)))]
              + tails[int(rng.integers(0, len(tails)))]} for _ in range(3000)]
    manifest = {"request.path": "STRING"}
    batch = BagBatch.from_bags(bags, names=list(manifest))
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    got, want = compare(eng, oracle.OracleEvaluator(manifest), rules, batch)
    assert all(0 < (want[:, j] == 1).sum() < batch.n for j in range(len(pats)))
    # the device path (deferred pairs, fused hit counters) agrees with the bitmaps' true bits
    import torch
    db = eng.upload(batch)
    Wd = (len(rules) + 31) // 32
    dm = torch.zeros((Wd, batch.n), dtype=torch.int32, device="cuda:0")
    flags_t = torch.zeros(batch.n, dtype=torch.uint8, device="cuda:0")
    hits = torch.zeros(len(rules), dtype=torch.int64, device="cuda:0")
    for _ in range(2):
        db.eval_compact(dm.data_ptr(), flags_t.data_ptr(), hits.data_ptr(), 0)
    torch.cuda.synchronize()
    assert np.array_equal(hits.cpu().numpy(), 2 * (want == 1).sum(axis=0))
    db.free()
