"""Parity at the BASELINE.json configuration sizes (VERDICT r1 "what's weak" #1).

* C3 (configs[2]): the full 100k-entry CIDR list on a 20k-lookup sample; 100k strings (and the
  case-insensitive variant) x 1M lookups; the full 10k-pattern regex union on 1000 lookups against
  the oracle, plus a 1M-lookup property (every lookup built to match some pattern is OK).
* C4 (configs[3]): all 10k route rules x 2048 requests against the oracle; and 10k x 1M with every
  routing the engine has -- value classes + prefix index (default), value classes off, guard index
  off -- bit-identical bitmaps.
* C2 at the bench size (10k x 1M): index on / off bit-identical.
* C2 and C4 exactly as bench.py evaluates them (10k x 1M, compact output + fused hit counters, and
  the bitmap output) against the oracle on a 4096-request sample, with error texts.
The oracle (oracle/lists.py, lists_oracle.c, il_interp.c + goregex.c) is the checker; the engine runs
through the C-ABI."""
import numpy as np
import pytest

import lists as L
import oracle
from istio_amd import workloads as W
from test_gpu_parity import compare

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mxp(libmxp):
    import istio_amd.engine as mxp
    return mxp


def test_c3_full_cidr_list(mxp):
    entries, syms = W.c3_ip_list(n_entries=100_000, n_lookups=20_000, seed=3)
    eng = mxp.Engine(0)
    lst = eng.list_create(L.IP_ADDRESSES, entries)
    ref = L.IPList(entries)
    assert lst.num_entries() == ref.num_entries() == 100_000
    for black in (False, True):
        want = L.codes(ref.found(syms, threads=16), black)
        got = lst.check(syms, black)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, [(syms[i], int(got[i]), int(want[i])) for i in bad[:5]]
    assert (want == 7).sum() > 5000 and (want == 0).sum() > 500  # (100k /8-/32 CIDRs cover most addresses)


@pytest.mark.parametrize("kind", [L.STRINGS, L.CASE_INSENSITIVE_STRINGS])
def test_c3_full_string_list(mxp, kind):
    entries, syms = W.c3_string_list(n_entries=100_000, n_lookups=1_000_000, seed=3)
    eng = mxp.Engine(0)
    lst = eng.list_create(kind, entries)
    ref = L.StringList(entries, case_insensitive=kind == L.CASE_INSENSITIVE_STRINGS)
    assert lst.num_entries() == ref.num_entries()
    want = L.codes(ref.found(syms), False)
    got = lst.check(syms)
    assert np.array_equal(got, want)
    assert (want == 0).sum() > 300_000 and (want == 5).sum() > 300_000


def test_c3_full_regex_union(mxp):
    pats, syms, hits = W.c3_regex_list(n_patterns=10_000, n_lookups=1_000_000, seed=3, return_hits=True)
    eng = mxp.Engine(0)
    lst = eng.list_create(L.REGEX, pats)
    assert lst.num_entries() == 10_000
    got = lst.check(syms)
    # every lookup built to match one of the patterns is found (whitelist: OK)
    assert (got[hits] == 0).all()
    # the oracle on a sample, all 10k patterns each
    sample = np.random.default_rng(9).choice(len(syms), 1000, replace=False)
    ref = L.RegexList(pats)
    want = L.codes(ref.found([syms[i] for i in sample], threads=16), False)
    bad = np.nonzero(got[sample] != want)[0]
    assert bad.size == 0, [(syms[sample[i]], int(got[sample[i]]), int(want[i])) for i in bad[:5]]
    assert (want == 0).sum() > 300 and (want == 5).sum() > 300


def test_c4_all_rules_against_oracle(mxp):
    manifest, rules, batch = W.c4_workload(n_rules=10_000, n_requests=2048, seed=4)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    got, want = compare(eng, oracle.OracleEvaluator(manifest), rules, batch)
    assert (want == 1).sum() > 2048 * 100


def _device_bitmaps(mxp, monkeypatch, flags, manifest, rules, batch):
    import torch
    monkeypatch.setenv("MXP_DEBUG_FLAGS", flags)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    db = eng.upload(batch)
    Wd = (len(rules) + 31) // 32
    dm = torch.empty((Wd, batch.n), dtype=torch.int32, device="cuda:0")
    de = torch.empty_like(dm)
    db.eval(dm.data_ptr(), de.data_ptr(), 0)
    torch.cuda.synchronize()
    db.free()
    return dm, de


@pytest.mark.parametrize("wl", ["c4", "c2"])
def test_full_size_routings_bit_identical(mxp, monkeypatch, wl):
    """10k rules x 1M requests: the optimised routings agree bit for bit with the plainest one."""
    import torch
    if wl == "c4":
        manifest, rules, batch = W.c4_workload(n_rules=10_000, n_requests=1 << 20, seed=4)
        variants = ["0", "131072", "8"]  # default (value classes + index), value classes off, index off
    else:
        manifest, rules, batch = W.c2_workload(n_rules=10_000, n_requests=1 << 20, seed=2)
        rules = W.c2_rules(10_000, seed=2)[0]
        variants = ["0", "8"]
    base = _device_bitmaps(mxp, monkeypatch, variants[-1], manifest, rules, batch)
    for flags in variants[:-1]:
        dm, de = _device_bitmaps(mxp, monkeypatch, flags, manifest, rules, batch)
        assert torch.equal(dm, base[0]) and torch.equal(de, base[1]), flags
        del dm, de
    assert int(torch.count_nonzero(base[0])) > 100_000


@pytest.mark.parametrize("wl", ["c2", "c4"])
def test_benched_evaluations_against_oracle(mxp, wl):
    """The evaluations bench.py times -- 10k rules x 1,048,576 requests, default routing, the compact
    output (match bitmap + per-request error flags) with fused hit counters, three steps back to back
    -- and the error-bitmap output, checked on a random 4096-request sample pair by pair against the
    oracle (not only routing against routing, which would miss a bug common to all routings); the hit
    counters against the bitmap; error texts of sampled error pairs from the host path's records."""
    import torch
    from istio_amd.engine import PANIC_TEXTS
    if wl == "c4":
        manifest, rules, batch = W.c4_workload(n_rules=10_000, n_requests=1 << 20, seed=4)
    else:
        manifest, rules, batch = W.c2_workload(n_rules=10_000, n_requests=1 << 20, seed=2)
        rules = W.c2_rules(10_000, seed=2)[0]
    R, N = len(rules), batch.n
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    db = eng.upload(batch)
    Wd = (R + 31) // 32
    s = torch.cuda.current_stream().cuda_stream
    dm = torch.zeros((Wd, N), dtype=torch.int32, device="cuda:0")
    req_err = torch.zeros(N, dtype=torch.uint8, device="cuda:0")
    hits = torch.zeros(R, dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()  # (the zeroing above is on torch's stream)
    for _ in range(3):
        db.eval_compact(dm.data_ptr(), req_err.data_ptr(), hits.data_ptr(), s)
    dm2 = torch.zeros_like(dm)
    de2 = torch.zeros_like(dm)
    db.eval(dm2.data_ptr(), de2.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(dm, dm2)
    # hit counters: 3 x the true pairs of each rule, counted from the bitmap here
    cnt = torch.zeros((Wd, 32), dtype=torch.int64, device="cuda:0")
    for b in range(32):
        cnt[:, b] = ((dm >> b) & 1).sum(dim=1)
    assert torch.equal(hits, 3 * cnt.reshape(-1)[:R])
    assert torch.equal(req_err.bool(), (de2 != 0).any(dim=0))
    rng = np.random.default_rng(17)
    sample = np.sort(rng.choice(N, 4096, replace=False))
    m = dm2[:, torch.from_numpy(sample).to("cuda:0")].cpu().numpy().view(np.uint32)
    e = de2[:, torch.from_numpy(sample).to("cuda:0")].cpu().numpy().view(np.uint32)
    db.free()
    del dm, dm2, de2, req_err, cnt
    torch.cuda.empty_cache()
    got = mxp.bits_to_codes(m, e, R)
    sub = batch.subset(sample)
    ev = oracle.OracleEvaluator(manifest)
    want = oracle.oracle_matrix(ev, rules, sub, threads=16)
    want_err = np.where(want >= 2, 2, want)
    bad = np.argwhere(got != want_err)
    assert bad.size == 0, [(int(sample[q]), int(r), int(got[q, r]), int(want_err[q, r])) for q, r in bad[:5]]
    assert (want == 1).sum() > 4096 * (0.3 if wl == "c2" else 100)
    # error texts: the host path over the whole batch (its bitmaps equal the device ones on the
    # sample), then the records of sampled error pairs
    hm, he = eng.eval_batch(batch)
    assert np.array_equal(hm[:, sample], m) and np.array_equal(he[:, sample], e)
    errs = np.argwhere(want >= 2)
    assert len(errs) > 0 or wl == "c4"  # (C4's routes have no error pairs)
    for q, r in errs[rng.choice(len(errs), min(300, len(errs)), replace=False)] if len(errs) else []:
        st, msg = ev.eval_predicate(rules[r], sub, int(q))
        gmsg = eng.pair_error(int(sample[q]), int(r))
        assert gmsg == msg or (st == "panic" and gmsg in PANIC_TEXTS), (rules[r], int(sample[q]), gmsg, msg)


def test_null_stream_orders_after_legacy_zeroing(mxp):
    """Round 3's race at bench size: counters and bitmaps zeroed by torch on the legacy default stream,
    then evaluations with stream=NULL and no host synchronisation in between -- libmxp's NULL stream
    must order after the zeroing (engine.cpp: a blocking stream), so the fused hit counters are exactly
    the bitmap's true pairs, three evaluations' worth, on C4 (value classes, deferred pairs)."""
    import torch
    manifest, rules, batch = W.c4_workload(n_rules=10_000, n_requests=1 << 20, seed=4)
    R, N = len(rules), batch.n
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    db = eng.upload(batch)
    Wd = (R + 31) // 32
    with torch.cuda.stream(torch.cuda.default_stream()):  # (earlier tests may leave another current)
        assert torch.cuda.current_stream().cuda_stream == 0  # torch's legacy default stream
        _null_stream_reps(db, R, N, Wd)
    db.free()


def _null_stream_reps(db, R, N, Wd):
    import torch
    dm = torch.full((Wd, N), -1, dtype=torch.int32, device="cuda:0")
    req_err = torch.full((N,), 7, dtype=torch.uint8, device="cuda:0")
    for rep in range(2):
        hits = torch.zeros(R, dtype=torch.int64, device="cuda:0")  # (no synchronize: stream order only)
        for _ in range(3):
            db.eval_compact(dm.data_ptr(), req_err.data_ptr(), hits.data_ptr(), 0)
        cnt = torch.zeros((Wd, 32), dtype=torch.int64, device="cuda:0")
        for b in range(32):
            cnt[:, b] = ((dm >> b) & 1).sum(dim=1)
        assert torch.equal(hits, 3 * cnt.reshape(-1)[:R]), rep
        assert int(hits.sum()) > 100 * N and int(req_err.max()) == 0


@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_c5_group_step(mxp, devices):
    """bench.py's C5 step on a device group (bench.group_step): every member's evaluation with fused
    hit counters, the memquota batch routed to its key owners on each member's second stream, and the
    step's one reduction -- three steps give 3 x the one-engine hit counters and exactly the per-key
    deltas of the sequential replay of the whole arrival stream (oracle/memquota.py restatement)."""
    import torch
    import bench
    import memquota as M
    from istio_amd.engine import key_owners
    manifest, rules, batch = W.c2_workload(n_rules=2000, n_requests=1 << 16, seed=2)
    R, N, K = len(rules), batch.n, bench.QUOTA_KEYS
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    db = eng.upload(batch)
    dm = torch.zeros(((R + 31) // 32, N), dtype=torch.int32, device="cuda:0")
    rq = torch.zeros(N, dtype=torch.uint8, device="cuda:0")
    h1 = torch.zeros(R, dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    db.eval_compact(dm.data_ptr(), rq.data_ptr(), h1.data_ptr(), 0)
    torch.cuda.synchronize()
    want_hits = h1.cpu().numpy().view(np.uint64)
    db.free()
    g = mxp.Group(devices)
    g.set_vocabulary(manifest)
    g.compile(rules)
    gb = g.upload(W.split_batch(batch, len(devices)))
    mx, vd, keys, amounts, be = W.quota_workload(n_keys=K, n_requests=N, seed=5)
    q = g.quota_create(mx, vd, key_owners(W.quota_key_weights(K), len(devices)))
    qb = q.upload(keys, amounts, be)
    now = [BASE_NS]
    step = bench.group_step(g, gb, (q, qb, now), g.stream(0))
    for _ in range(3):
        step()
    hits, delta = g.counters(K)
    ref = M.CMemquota(mx, vd)
    want_delta = np.zeros(K, dtype=np.int64)
    for s in range(3):
        np.add.at(want_delta, keys.astype(np.int64),
                  np.sign(amounts) * ref.handle_batch(keys, amounts, be, BASE_NS + s * 10**8, threads=16))
    assert np.array_equal(hits, 3 * want_hits) and int(hits.sum()) > 0
    assert np.array_equal(delta, want_delta) and (delta != 0).any()
    qb.free()
    gb.free()


BASE_NS = 1_500_000_000 * 10**9


@pytest.mark.parametrize("wl", ["c4", "c2"])
def test_recycled_batch_blocks_match_fresh_engine(mxp, wl):
    """mxp_batch_free hands a batch's device blocks to the engine's bin and later uploads reuse them
    (engine_impl.h BlockBin): batches uploaded into recycled blocks -- a larger batch's, holding its
    stale words, and, shrinking, blocks larger than asked for -- evaluate bit for bit as the same
    batches uploaded by a fresh engine, with evaluations still in flight on another stream when the
    blocks are freed."""
    import torch
    sizes = [(1 << 17) + 5, 50_001, 3_000]
    if wl == "c4":
        mk = lambda n, seed: W.c4_workload(n_rules=2000, n_requests=n, seed=seed)
    else:
        mk = lambda n, seed: W.c2_workload(n_rules=2000, n_requests=n, seed=seed)
    batches = [mk(n, 40 + k) for k, n in enumerate(sizes)]
    manifest, rules = batches[0][0], batches[0][1]
    if wl == "c2":
        rules = W.c2_rules(2000, seed=2)[0]
    Wd = (len(rules) + 31) // 32

    def run(eng, b, s, free_after=True):
        db = eng.upload(b)
        dm = torch.zeros((Wd, b.n), dtype=torch.int32, device="cuda:0")
        de = torch.zeros_like(dm)
        db.eval(dm.data_ptr(), de.data_ptr(), s.cuda_stream)
        if free_after:
            db.free()  # (the evaluation may still be running on s)
        return dm, de

    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    s = torch.cuda.Stream()
    got = [run(eng, b[2], s) for b in batches]            # each upload draws the previous one's blocks
    got += [run(eng, b[2], s) for b in reversed(batches)]  # and growing again
    torch.cuda.synchronize()
    ref_eng = mxp.Engine(0)
    ref_eng.set_vocabulary(manifest)
    ref_eng.compile(rules)
    for k, b in enumerate(list(batches) + list(reversed(batches))):
        dm, de = run(ref_eng, b[2], s)
        torch.cuda.synchronize()
        assert torch.equal(got[k][0], dm) and torch.equal(got[k][1], de), (wl, k)
    assert int(torch.count_nonzero(got[0][0])) > 1000
