"""Device groups (include/mxp_group.h): the multi-GPU engine a Go Mixer drives from one process.

* A group over [0] with its one-rank RCCL all-reduce (MXP_GROUP_RCCL_SINGLE) evaluates C2 and C4 at
  the bench size (10k rules x 1M requests) bit for bit as one engine does, its counters (fused hit
  counters, all-reduced, folded into the totals) equal to the bitmap's true pairs, and a 4096-request
  sample against the oracle.
* A group of two members on device 0 (RCCL refuses two ranks on one GPU, so the host reduction runs)
  splits the batch into contiguous shards whose concatenated bitmaps equal the one-engine bitmaps,
  with exact summed hit counters.
* memquota routed to key owners inside the group replays each key's sequence exactly as the
  sequential restatement (oracle/memquota.py) does for the whole arrival stream, with the per-key
  deltas all-reduced into the counters.
* Resolve, list checks and a finder vocabulary over the group equal the one-engine results.
* A group larger than its batch (members with 0 or 1 requests) evaluates and resolves as one engine."""
import numpy as np
import pytest

import memquota as M
import oracle
from istio_amd import workloads as W

pytestmark = pytest.mark.gpu
BASE_NS = 1_500_000_000 * 10**9


@pytest.fixture(scope="module")
def mxp(libmxp):
    import istio_amd.engine as mxp
    return mxp


def _workload(wl, n_rules, n_requests):
    if wl == "c4":
        return W.c4_workload(n_rules=n_rules, n_requests=n_requests, seed=4)
    manifest, _, batch = W.c2_workload(n_rules=n_rules, n_requests=n_requests, seed=2)
    return manifest, W.c2_rules(n_rules, seed=2)[0], batch


def _engine_reference(mxp, manifest, rules, batch):
    """One engine's compact evaluation of the whole batch: (match bitmap, request error flags, hits)."""
    import torch
    R, N = len(rules), batch.n
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    db = eng.upload(batch)
    Wd = (R + 31) // 32
    dm = torch.zeros((Wd, N), dtype=torch.int32, device="cuda:0")
    rq = torch.zeros(N, dtype=torch.uint8, device="cuda:0")
    hits = torch.zeros(R, dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    db.eval_compact(dm.data_ptr(), rq.data_ptr(), hits.data_ptr(), 0)
    torch.cuda.synchronize()
    out = dm.cpu().numpy().view(np.uint32), rq.cpu().numpy(), hits.cpu().numpy().view(np.uint64)
    db.free()
    eng.close()
    return out


def _bit_counts(match, R):
    cnt = np.zeros(match.shape[0] * 32, dtype=np.uint64)
    for b in range(32):
        cnt[b::32] = ((match >> np.uint32(b)) & 1).sum(axis=1)
    return cnt[:R]


@pytest.mark.parametrize("wl", ["c2", "c4"])
def test_single_member_rccl_matches_engine(mxp, wl):
    manifest, rules, batch = _workload(wl, 10_000, 1 << 20)
    R, N = len(rules), batch.n
    ref_m, ref_e, ref_h = _engine_reference(mxp, manifest, rules, batch)
    g = mxp.Group([0], mxp.GROUP_RCCL_SINGLE)
    assert g.reduce_mode == mxp.REDUCE_RCCL, g.note
    g.set_vocabulary(manifest)
    assert (g.compile(rules) == 0).all()
    gb = g.upload([batch])
    steps = 3
    for _ in range(steps):
        g.eval(gb)
        g.reduce()
    hits, _ = g.counters()
    m, e = g.download(0, N)
    assert np.array_equal(m, ref_m) and np.array_equal(e, ref_e)
    assert np.array_equal(hits, steps * ref_h)
    assert np.array_equal(hits, steps * _bit_counts(m, R)) and int(hits.sum()) > N // 4
    # the oracle on a sample of the group's own bitmap (error-bitmap form)
    g.eval(gb, err_bitmap=True)
    m2, e2 = g.download(0, N, err_bitmap=True)
    assert np.array_equal(m2, m) and np.array_equal((e2 != 0).any(axis=0).astype(np.uint8), e)
    sample = np.sort(np.random.default_rng(23).choice(N, 4096, replace=False))
    got = mxp.bits_to_codes(m2[:, sample], e2[:, sample], R)
    want = oracle.oracle_matrix(oracle.OracleEvaluator(manifest), rules, batch.subset(sample), threads=16)
    bad = np.argwhere(got != np.where(want >= 2, 2, want))
    assert bad.size == 0, bad[:5]
    gb.free()
    g.close()


@pytest.mark.parametrize("wl", ["c2", "c4"])
def test_two_members_host_reduce_bit_identical(mxp, wl):
    manifest, rules, batch = _workload(wl, 10_000, 1 << 20)
    R, N = len(rules), batch.n
    ref_m, ref_e, ref_h = _engine_reference(mxp, manifest, rules, batch)
    g = mxp.Group([0, 0])
    assert g.reduce_mode == mxp.REDUCE_HOST and "twice" in g.note
    g.set_vocabulary(manifest)
    assert (g.compile(rules) == 0).all()
    gb = g.upload_split(batch)
    assert gb.counts == [N // 2, N - N // 2]
    for _ in range(2):
        g.eval(gb)
        g.reduce()
    hits, _ = g.counters()
    parts = [g.download(k, gb.counts[k]) for k in range(2)]
    assert np.array_equal(np.concatenate([p[0] for p in parts], axis=1), ref_m)
    assert np.array_equal(np.concatenate([p[1] for p in parts]), ref_e)
    assert np.array_equal(hits, 2 * ref_h)
    assert g.locate(N // 2) == (1, 0) and g.locate(N // 2 - 1) == (0, N // 2 - 1)
    gb.free()
    g.close()


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
def test_quota_routed_to_owners(mxp, devices):
    """Owner routing inside the group: three batches of 200k requests at advancing times, granted
    amounts in arrival order and per-key deltas (summed over the members by the reduction) equal the
    sequential replay of the whole stream."""
    K = 1024
    mx, vd, keys, amounts, be = W.quota_workload(n_keys=K, n_requests=600_000, seed=61)
    g = mxp.Group(devices)
    owner = mxp.key_owners(W.quota_key_weights(K), len(devices))
    q = g.quota_create(mx, vd, owner)
    ref = M.CMemquota(mx, vd)
    want_delta = np.zeros(K, dtype=np.int64)
    now = BASE_NS
    for b in range(3):
        sl = slice(b * 200_000, (b + 1) * 200_000)
        qb = q.upload(keys[sl], amounts[sl], be[sl])
        assert sum(qb.requests(k) for k in range(len(devices))) == 200_000
        for k in range(len(devices)):  # every member got exactly its own keys' requests
            assert qb.requests(k) == int((owner[keys[sl]] == k).sum())
        q.eval(qb, now)
        g.reduce()
        got = qb.granted()
        want = ref.handle_batch(keys[sl], amounts[sl], be[sl], now, threads=16)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (b, bad[:5])
        np.add.at(want_delta, keys[sl].astype(np.int64), np.sign(amounts[sl]) * want)  # allocs - frees
        qb.free()
        now += [400_000_000, 3 * 10**9, 61 * 10**9][b]
    _, delta = g.counters(K)
    assert np.array_equal(delta, want_delta) and (want_delta != 0).any()
    del q
    g.close()


def test_key_owners_match_dist(mxp):
    from istio_amd import dist as D
    for n in (1, 2, 3, 8):
        w = W.quota_key_weights(1024)
        assert np.array_equal(mxp.key_owners(w, n), D.key_owners(w, n))


def test_resolve_over_group_matches_engine(mxp):
    """mxp_group_resolve_batch over three members (shards of one batch) returns exactly what one
    engine's mxp_resolve_batch returns for the whole batch: statuses, first-error rules, action
    lists (both id widths) and the error texts of failing requests."""
    manifest, rules, batch = W.c2_workload(n_rules=3000, n_requests=200_003, seed=2)
    rules = W.c2_rules(3000, seed=2)[0]
    R = len(rules)
    ns = ["istio-system"] * (R // 2) + ["ns%d" % (i % 8) for i in range(R - R // 2)]
    order = np.argsort(np.array(ns, dtype=object), kind="stable")
    rules = [rules[i] for i in order]
    ns = [ns[i] for i in order]
    vm = (np.arange(R) % 3 + 1).astype(np.uint32)
    tcp = (np.arange(R) % 11 == 0).astype(np.uint8)
    empty = (np.arange(R) % 13 == 0).astype(np.uint8)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    eng.set_resolver("destination.service", "istio-system", ns, vm, tcp, empty)
    g = mxp.Group([0, 0, 0])
    g.set_vocabulary(manifest)
    g.compile(rules)
    g.set_resolver("destination.service", "istio-system", ns, vm, tcp, empty)
    view = W.split_batch(batch, 3)
    for variety in (0, 1):
        for ids16 in (False, True):
            s1, e1, o1, r1 = eng.resolve_arrays(batch, variety, ids16=ids16)
            s2, e2, o2, r2 = g.resolve_arrays(view, variety, ids16=ids16)
            assert np.array_equal(s1, s2) and np.array_equal(o1, o2) and np.array_equal(r1, r2)
            err = np.nonzero(s1 == 3)[0]
            assert np.array_equal(e1[err], e2[err])
    assert len(err) > 0 and len(r1) > batch.n // 10
    for q in err[:: max(1, len(err) // 50)]:
        assert g.pair_error(int(q), int(e2[q])) == eng.pair_error(int(q), int(e1[q]))


def test_lists_over_group(mxp):
    import lists as L
    entries, syms = W.c3_ip_list(n_entries=20_000, n_lookups=100_001, seed=3)
    eng = mxp.Engine(0)
    want = eng.list_create(L.IP_ADDRESSES, entries).check(syms, True)
    g = mxp.Group([0, 0])
    gl = g.list_create(L.IP_ADDRESSES, entries)
    assert np.array_equal(gl.check(syms, True), want)
    pats, rsyms = W.c3_regex_list(n_patterns=2000, n_lookups=50_000, seed=3)
    want = eng.list_create(L.REGEX, pats).check(rsyms)
    assert np.array_equal(g.list_create(L.REGEX, pats).check(rsyms), want)


def test_finder_vocabulary_over_group(mxp):
    """mxp_group_vocab_set_finder: the finder is asked on the calling thread only, each name once, and
    every member compiles (statuses, hit counters) as with the whole manifest."""
    manifest, rules, batch = W.c2_workload(n_rules=500, n_requests=20_000, seed=2)
    rules = W.c2_rules(500, seed=2)[0] + ["nope == 2"]
    asked = []

    def get_attribute(name):
        asked.append(name)
        return manifest.get(name)
    g = mxp.Group([0, 0])
    g.set_vocabulary_finder(get_attribute)
    st = g.compile(rules)
    assert st[-1] == mxp.RULE_TYPE_ERROR and (st[:-1] == 0).all()
    assert len(asked) == len(set(asked)) and "nope" in asked
    gb = g.upload_split(batch)
    g.eval(gb)
    g.reduce()
    hits, _ = g.counters()
    h = mxp.Group([0])
    h.set_vocabulary(manifest)
    h.compile(rules)
    hb = h.upload([batch])
    h.eval(hb)
    h.reduce()
    assert np.array_equal(hits, h.counters()[0]) and hits.sum() > 0


@pytest.mark.parametrize("devices", [None, [0, 0]])
@pytest.mark.parametrize("split", [False, True])
def test_resolve_uploaded_pipeline(mxp, devices, split):
    """mxp_resolve_uploaded / mxp_group_resolve_uploaded: batch k + 1 uploaded (MXP_UPLOAD_NO_WAIT)
    before batch k is resolved -- as bench.py's pipelined end-to-end figure and a double-buffering
    micro-batcher do -- gives each batch exactly the plain Resolve's statuses, first-error rules,
    action lists and error texts.  split: the two-call Resolve (mxp_resolve_submit / _finish), batch
    k + 1 uploaded between batch k's submit and finish."""
    manifest, _, _ = W.c2_workload(n_rules=1500, n_requests=1, seed=2)
    rules = W.c2_rules(1500, seed=2)[0]
    R = len(rules)
    ns, vm = ["istio-system"] * R, np.ones(R, dtype=np.uint32)
    z = np.zeros(R, dtype=np.uint8)
    batches = [W.c2_workload(n_rules=1500, n_requests=3 * 90_001, seed=2, shard=(k * 90_001, (k + 1) * 90_001))[2]
               for k in range(3)]
    ref = mxp.Engine(0)
    ref.set_vocabulary(manifest)
    ref.compile(rules)
    ref.set_resolver("destination.service", "istio-system", ns, vm, z, z)
    want = [ref.resolve_arrays(b, 0, ids16=True) for b in batches]
    texts = []
    for b, w in zip(batches, want):
        ref.resolve_arrays(b, 0, ids16=True)
        err = np.nonzero(w[0] == 3)[0][:40]
        texts.append([ref.pair_error(int(q), int(w[1][q])) for q in err])
    assert sum(len(t) for t in texts) > 0
    if devices is None:
        eng = mxp.Engine(0)
        eng.set_vocabulary(manifest)
        eng.compile(rules)
        eng.set_resolver("destination.service", "istio-system", ns, vm, z, z)
        nxt = eng.upload(batches[0], no_wait=True)
        for k, b in enumerate(batches):
            cur = nxt
            job = eng.resolve_submit(cur, 0, ids16=True) if split else None
            if k + 1 < len(batches):
                nxt = eng.upload(batches[k + 1], no_wait=True)
            got = eng.resolve_finish(job, 1 << 22) if split else eng.resolve_uploaded(cur, 0, cap=1 << 22, ids16=True)
            for a, c in zip(got, want[k]):
                assert np.array_equal(a, c), k
            err = np.nonzero(want[k][0] == 3)[0][:40]
            assert [eng.pair_error(int(q), int(got[1][q])) for q in err] == texts[k]
        return
    g = mxp.Group(devices)
    g.set_vocabulary(manifest)
    g.compile(rules)
    g.set_resolver("destination.service", "istio-system", ns, vm, z, z)
    shards = [W.split_batch(b, len(devices)) for b in batches]
    nxt = g.upload(shards[0], no_wait=True)
    for k in range(len(batches)):
        cur = nxt
        job = g.resolve_submit(cur, 0, ids16=True) if split else None
        if k + 1 < len(batches):
            nxt = g.upload(shards[k + 1], no_wait=True)
        got = (g.resolve_finish(job, 1 << 22) if split
               else g.resolve_arrays(shards[k], 0, cap=1 << 22, ids16=True, uploaded=cur))
        for a, c in zip(got, want[k]):
            assert np.array_equal(a, c), k
        err = np.nonzero(want[k][0] == 3)[0][:40]
        assert [g.pair_error(int(q), int(got[1][q])) for q in err] == texts[k]


@pytest.mark.parametrize("n", [1, 2, 5, 1000])
def test_group_members_with_few_or_no_requests(mxp, n):
    """A batch smaller than the group (members with 0 or 1 requests): three members on device 0
    evaluate (bitmaps, request error flags, summed hit counters) and resolve exactly as one engine
    does over the whole batch."""
    manifest, rules, full = _workload("c2", 2000, 4096)
    batch = full.subset(np.arange(n))
    R = len(rules)
    ref_m, ref_e, ref_h = _engine_reference(mxp, manifest, rules, batch)
    g = mxp.Group([0, 0, 0])
    g.set_vocabulary(manifest)
    assert (g.compile(rules) == 0).all()
    gb = g.upload_split(batch)
    assert sum(gb.counts) == n and len(gb.counts) == 3
    g.eval(gb)
    g.reduce()
    hits, _ = g.counters()
    parts = [g.download(k, gb.counts[k]) for k in range(3) if gb.counts[k]]
    assert np.array_equal(np.concatenate([p[0] for p in parts], axis=1), ref_m)
    assert np.array_equal(np.concatenate([p[1] for p in parts]), ref_e)
    assert np.array_equal(hits, ref_h)
    gb.free()
    ns = ["istio-system"] * R
    vm = np.ones(R, dtype=np.uint32)
    zero = np.zeros(R, dtype=np.uint8)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    eng.set_resolver("destination.service", "istio-system", ns, vm, zero, zero)
    g.set_resolver("destination.service", "istio-system", ns, vm, zero, zero)
    s1, e1, o1, r1 = eng.resolve_arrays(batch, 0, ids16=True)
    s2, e2, o2, r2 = g.resolve_arrays(W.split_batch(batch, 3), 0, ids16=True)
    m = int(o1[-1])
    assert np.array_equal(s1, s2) and np.array_equal(o1, o2) and np.array_equal(r1[:m], r2[:m])
    err = np.nonzero(s1 == 3)[0]
    assert np.array_equal(e1[err], e2[err])
    eng.close()
    g.close()
