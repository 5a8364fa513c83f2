"""Pair Resolve (resolve.hip resolve_pairs): when every word of the rule set is a plain fill chunk's
(C2's ==/startsWith/ip() rules), a Resolve reads the evaluation's deferred index pairs, filed per
fill chunk and lane quad, instead of a match bitmap the evaluation then never writes
(kargs.dtp_lazy).  Bar: status, first-error rule, offsets and rule ids identical to the bitmap
Resolve (MXP_RESOLVE_PAIRS=0, itself pinned against the resolver restatement in
test_gpu_resolver.py) and to the restatement (oracle/resolver.py over the oracle's codes) on a
small batch -- with namespaces before and after the default one in rule order, varieties, TCP
flags, missing identities and predicate errors; pairs past their lists (MXP_DTP_CAP=4) fall back to
the bitmap the fills then store.  MXP_RESOLVE_PAIRS=2 makes a Resolve that cannot take the pair
path fail, so these tests know it ran."""
import numpy as np
import pytest

import oracle
import resolver as oracle_resolver
from istio_amd import workloads as W
from istio_amd.bags import ABSENT, STRING, BagBatch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mxp(libmxp):
    import istio_amd.engine as mxp
    return mxp


def c2_resolve_case(n_base, copies, n_requests, seed):
    """C2 requests over n_base C2 rules, plus a context.protocol column (tcp / http / missing) and 0.2 %
    of the identities missing; the rule set is four namespace blocks in rule order ns1, ns0 (the
    default), ns2, ns5 (the batch's destinations name ns0 .. ns7), each block the n_base rules
    `copies` times over (copies n_base rules apart: a request matching one rule selects every copy
    in both of its namespaces)."""
    manifest, base, b = W.c2_workload(n_rules=n_base, n_requests=n_requests, seed=seed)
    # (copy j compares source.ip with an address outside 10/8, where the requests' are: the same
    # pairs, but a program of its own -- eight byte-identical rules would become a dense id)
    block = [r.replace('ip("10.', 'ip("%d.' % (10 + j)) for j in range(copies) for r in base]
    rules = block * 4
    n_rules = len(rules)
    rng = np.random.default_rng(seed + 7)
    n = b.n
    strings = [b.string(i) for i in range(b.n_strings)] + [b"tcp", b"http"]
    offs = np.zeros(len(strings) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(s) for s in strings])
    blob = np.frombuffer(b"".join(strings) + b"\0", dtype=np.uint8).copy()
    r = rng.random(n)
    pk = np.where(r < 0.9, STRING, ABSENT).astype(np.uint8)
    pv = np.where(r < 0.3, len(strings) - 2, len(strings) - 1).astype(np.uint64)
    kinds = [k.copy() for k in b.kinds]
    di = b.names.index("destination.service")
    kinds[di][rng.random(n) < 0.002] = ABSENT  # (every rule errors there: few, so records fit the log)
    batch = BagBatch(n, b.names + ["context.protocol"], kinds + [pk], b.values + [pv], blob, offs)
    q = n_rules // 4
    rule_ns = ["ns1"] * q + ["ns0"] * q + ["ns2"] * q + ["ns5"] * (n_rules - 3 * q)
    conf = dict(rule_ns=rule_ns, variety_mask=[int(x) for x in rng.integers(1, 16, size=n_rules)],
                is_tcp=[int(x) for x in rng.random(n_rules) < 0.3], empty_match=[0] * n_rules,
                identity_attr="destination.service", default_ns="ns0")
    return manifest, rules, conf, batch


def engine_for(mxp, monkeypatch, manifest, rules, conf, pairs, extra=None):
    monkeypatch.setenv("MXP_RESOLVE_PAIRS", pairs)
    for k, v in (extra or {}).items():
        monkeypatch.setenv(k, v)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    eng.set_resolver(conf["identity_attr"], conf["default_ns"], conf["rule_ns"], conf["variety_mask"],
                     conf["is_tcp"], conf["empty_match"])
    return eng


def test_pair_resolve_matches_restatement(mxp, monkeypatch):
    manifest, rules, conf, batch = c2_resolve_case(512, 1, 1024, seed=31)
    eng = engine_for(mxp, monkeypatch, manifest, rules, conf, "2")
    ev = oracle.OracleEvaluator(manifest)
    codes = oracle.oracle_matrix(ev, rules, batch, threads=16)
    seen = set()
    for variety in (0, 1, 3):
        status, err_rule, sel = eng.resolve(batch, variety)
        want = oracle_resolver.resolve(batch, codes, conf["rule_ns"], conf["variety_mask"], conf["is_tcp"],
                                       conf["empty_match"], conf["identity_attr"], conf["default_ns"], variety)
        for q, (ws, we, wsel) in enumerate(want):
            assert status[q] == ws, (q, variety, status[q], ws)
            seen.add(ws)
            if ws == oracle_resolver.PRED_ERROR:
                assert err_rule[q] == we, (q, variety)
            else:
                assert list(sel[q]) == wsel, (q, variety)
    assert {0, 1, 3} <= seen
    eng.close()


@pytest.mark.parametrize("extra", [{}, {"MXP_DTP_CAP": "4"}], ids=["pairs", "overflow"])
def test_pair_resolve_equals_bitmap(mxp, monkeypatch, extra):
    """~10k rules (833 C2 rules three times in each of four namespaces) over 128k requests: the pair Resolve (required unless pairs overflow) equals the
    bitmap Resolve in every output, u16 and u32 ids, three varieties; more than four rules for some
    requests (the write pass's walk) and for most at most four (the stash)."""
    manifest, rules, conf, batch = c2_resolve_case(833, 3, 131072, seed=32)
    got = {}
    for pairs in ("2" if not extra else "1", "0"):
        eng = engine_for(mxp, monkeypatch, manifest, rules, conf, pairs, extra)
        got[pairs] = [[x.copy() for x in eng.resolve_arrays(batch, v, ids16=u16)] for v in (0, 2, 5)
                      for u16 in (False, True)]
        eng.close()
    a_key = "2" if not extra else "1"
    for a, b in zip(got[a_key], got["0"]):
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
    st, _, off, _ = got["0"][0]
    counts = np.diff(off.astype(np.int64))
    assert (st == 0).sum() > 50000 and (st == 3).sum() > 100 and (st == 1).sum() > 100
    assert counts.max() > 4 and int(off[-1]) > 10000


def test_pair_resolve_group_pipeline(mxp, monkeypatch):
    """The group's two-call Resolve over uploaded narrow shards takes the pair path (required) and
    equals the one-engine bitmap Resolve of the whole batch."""
    manifest, rules, conf, batch = c2_resolve_case(520, 1, 65536, seed=33)
    eng = engine_for(mxp, monkeypatch, manifest, rules, conf, "0")
    want = [x.copy() for x in eng.resolve_arrays(batch, 1, ids16=True)]
    eng.close()
    monkeypatch.setenv("MXP_RESOLVE_PAIRS", "2")
    g = mxp.Group([0, 0])
    g.set_vocabulary(manifest)
    g.compile(rules)
    g.set_resolver(conf["identity_attr"], conf["default_ns"], conf["rule_ns"], conf["variety_mask"],
                   conf["is_tcp"], conf["empty_match"])
    shards = W.split_batch(batch, 2)
    cap = 4 * batch.n
    for _ in range(2):
        up = g.upload(shards, no_wait=True)
        job = g.resolve_submit(up, 1, ids16=True)
        status, err_rule, off, ids = g.resolve_finish(job, cap)
        assert np.array_equal(status, want[0]) and np.array_equal(err_rule, want[1])
        assert np.array_equal(off, want[2]) and np.array_equal(ids[:int(off[-1])], want[3][:int(want[2][-1])])
    g.close()


def test_resolver_tables_follow_configuration(mxp, monkeypatch):
    """The resolver's per-word tables stay on the device between calls of one configuration and
    variety; a new configuration (mxp_resolver_set) or variety replaces them: an engine re-configured
    between calls resolves as a fresh engine with the new configuration."""
    manifest, rules, conf, batch = c2_resolve_case(512, 1, 8192, seed=34)
    conf2 = dict(conf, variety_mask=[int(x) ^ 5 for x in conf["variety_mask"]],
                 is_tcp=[1 - int(x) for x in conf["is_tcp"]], default_ns="ns2")
    eng = engine_for(mxp, monkeypatch, manifest, rules, conf, "1")
    fresh = engine_for(mxp, monkeypatch, manifest, rules, conf2, "1")
    a = [x.copy() for x in eng.resolve_arrays(batch, 1)]
    b = [x.copy() for x in eng.resolve_arrays(batch, 2)]
    eng.set_resolver(conf2["identity_attr"], conf2["default_ns"], conf2["rule_ns"], conf2["variety_mask"],
                     conf2["is_tcp"], conf2["empty_match"])
    for v in (1, 2, 1):
        got, want = eng.resolve_arrays(batch, v), fresh.resolve_arrays(batch, v)
        for x, y in zip(got, want):
            assert np.array_equal(x, y), v
    assert not all(np.array_equal(x, y) for x, y in zip(a, b))
    eng.close()
    fresh.close()


@pytest.mark.parametrize("pairs", ["1", "0"])
def test_ids_enqueued_with_outputs(mxp, monkeypatch, pairs):
    """Pinned outputs: the ids are written (guarded by the capacity) and downloaded with the other
    outputs before the host knows their count.  Exact, larger and too-small capacities (the latter
    returns MXP_ERR_NOMEM with sel_off complete, and resolve_arrays retries) give the pageable
    call's outputs -- one engine, and a group's first member (its ids go first in the list)."""
    from istio_amd.engine import PinnedArena
    manifest, rules, conf, batch = c2_resolve_case(520, 2, 32768, seed=35)
    eng = engine_for(mxp, monkeypatch, manifest, rules, conf, pairs)
    for u16 in (False, True):
        want = [x.copy() for x in eng.resolve_arrays(batch, 1, ids16=u16)]
        total = int(want[2][-1])
        assert total > 100
        for cap in (total, total + 1000, total - 1, 16):
            got = eng.resolve_arrays(batch, 1, cap=cap, ids16=u16, pinned=True)
            for x, y in zip(got, want):
                assert np.array_equal(x, y), (u16, cap)
    eng.close()
    g = mxp.Group([0, 0])
    g.set_vocabulary(manifest)
    g.compile(rules)
    g.set_resolver(conf["identity_attr"], conf["default_ns"], conf["rule_ns"], conf["variety_mask"],
                   conf["is_tcp"], conf["empty_match"])
    shards = W.split_batch(batch, 2)
    want = [x.copy() for x in g.resolve_arrays(shards, 1, ids16=True)]
    total, n = int(want[2][-1]), batch.n
    for cap in (total, total + 64):
        arena = PinnedArena(n * 13 + 8 + cap * 2 + 4 * 64)
        out = (arena.empty(n, np.uint8), arena.empty(n, np.uint32), arena.empty(n + 1, np.uint64),
               arena.empty(cap, np.uint16))
        got = g.resolve_arrays(shards, 1, cap=cap, ids16=True, out=out)
        for x, y in zip(got, want):
            assert np.array_equal(x, y), cap
        job = g.resolve_submit(g.upload(shards, no_wait=True), 1, ids16=True)
        got = g.resolve_finish(job, cap, out=out)
        for x, y in zip(got, want):
            assert np.array_equal(x, y), cap
    g.close()


@pytest.mark.parametrize("n", [0, 1, 3, 5, 1000, 1025, 4097, 66001])
def test_pair_resolve_ragged_batches(mxp, monkeypatch, n):
    """Batch sizes that are not multiples of the pair passes' quad (4 requests), tile (1,024) or
    index wave (64): the pair Resolve (required for n > 0) equals the bitmap Resolve in every output,
    one engine and a two-member group over the same GPU (contiguous shards, mxp_group_shard_bounds)."""
    manifest, rules, conf, full = c2_resolve_case(520, 2, 66001 + 7, seed=36)
    batch = full.subset(np.arange(7, 7 + n))
    got = {}
    for pairs in ("2" if n else "1", "0"):
        eng = engine_for(mxp, monkeypatch, manifest, rules, conf, pairs)
        got[pairs] = [x.copy() for x in eng.resolve_arrays(batch, 1, ids16=True)]
        eng.close()
    a = got["2" if n else "1"]
    for x, y in zip(a, got["0"]):
        assert np.array_equal(x, y), n
    assert len(a[0]) == n and len(a[2]) == n + 1
    if n >= 1000:
        assert int(a[2][-1]) > 0 and (a[0] == 3).sum() + (a[0] == 1).sum() > 0
    if n >= 2:
        monkeypatch.setenv("MXP_RESOLVE_PAIRS", "2")
        g = mxp.Group([0, 0])
        g.set_vocabulary(manifest)
        g.compile(rules)
        g.set_resolver(conf["identity_attr"], conf["default_ns"], conf["rule_ns"], conf["variety_mask"],
                       conf["is_tcp"], conf["empty_match"])
        shards = W.split_batch(batch, 2)
        assert sum(s.n for s in shards) == n and min(s.n for s in shards) >= 1
        st, er, off, ids = g.resolve_arrays(shards, 1, ids16=True)
        want = got["0"]
        assert np.array_equal(st, want[0]) and np.array_equal(er, want[1]) and np.array_equal(off, want[2]), n
        m = int(want[2][-1])
        assert np.array_equal(ids[:m], want[3][:m]), n
        g.close()
