"""Deferred index pairs (kernels.hip "Deferred pairs", engine.cpp launch): with value classes active
and every indexed group written by the value-class fill, the guard-index kernel runs first and
records its true / error pairs per wave; mxp_dtp_sort_kernel orders them by (fill chunk, lane
quad) and mxp_vtfill_*_kernel ORs them into the words it writes.  Pairs past a wave's capacity go
to an overflow list OR-ed in after the fill; past that list's capacity the index kernel re-runs
with plain OR-s.  Bar: bit-exact against the oracle (error texts included) and against the
engine with deferred pairs off (MXP_DTP=0), on every one of those three paths."""
import numpy as np
import pytest

import oracle
from istio_amd import workloads as W
from test_gpu_parity import compare

pytestmark = pytest.mark.gpu
FORCE = "262144"  # value classes at any batch size


@pytest.fixture(scope="module")
def mxp(libmxp):
    import istio_amd.engine as mxp
    return mxp


def engine_for(mxp, monkeypatch, env, manifest, rules, flags=FORCE):
    for k in ("MXP_DTP", "MXP_DTP_CAP", "MXP_DTP_OVF"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("MXP_DEBUG_FLAGS", flags)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    return eng


def deferred_ran(eng, batch, R):
    """Whether a device evaluation of `batch` takes the deferred-pair path (mxp_kernel_times [2])."""
    import torch
    db = eng.upload(batch)
    dm = torch.zeros(((R + 31) // 32, batch.n), dtype=torch.int32, device="cuda:0")
    de = torch.zeros_like(dm)
    hits = torch.zeros(R, dtype=torch.int64, device="cuda:0")
    eng.set_timing(True)
    db.eval_hits(dm.data_ptr(), de.data_ptr(), hits.data_ptr(), 0)
    t = eng.kernel_times(3)
    eng.set_timing(False)
    db.free()
    return len(t) == 3 and t[2] == 1.0


# default capacity; 4 pairs per wave (most go to the overflow list); 4 per wave and an overflow
# list of 8 (full: the gated index re-run ORs every pair)
PATHS = [{}, {"MXP_DTP_CAP": "4"}, {"MXP_DTP_CAP": "4", "MXP_DTP_OVF": "8"}]


@pytest.mark.parametrize("env", PATHS, ids=["lists", "overflow", "rerun"])
def test_deferred_pairs_parity(mxp, monkeypatch, env):
    """C4 routes with continuations (`path.startsWith(p) && source.ip == ip(..)`, source.ip absent
    for 30%): true and lookup-error pairs from the index kernel, a ragged batch."""
    manifest, rules, batch = W.c4_workload(n_rules=1500, n_requests=8000 + 13, seed=47, cont_frac=0.5)
    eng = engine_for(mxp, monkeypatch, env, manifest, rules)
    assert deferred_ran(eng, batch, len(rules))
    got, want = compare(eng, oracle.OracleEvaluator(manifest), rules, batch, sample_msgs=300)
    cont = [i for i, r in enumerate(rules) if "source.ip" in r]
    assert (want[:, cont] == 1).sum() > 50 and (want[:, cont] >= 2).sum() > 50


def test_deferred_pairs_device_identical(mxp, monkeypatch):
    """Device bitmaps and hit counters (fused and streamed), bitmap and compact error output:
    deferred pairs on (each of the three paths) equal deferred pairs off."""
    import torch
    manifest, rules, batch = W.c4_workload(n_rules=2000, n_requests=50_000 + 5, seed=48, cont_frac=0.3)
    Wd = (len(rules) + 31) // 32
    out = []
    for env in PATHS + [{"MXP_DTP": "0"}]:
        eng = engine_for(mxp, monkeypatch, env, manifest, rules)
        assert deferred_ran(eng, batch, len(rules)) == (env.get("MXP_DTP") != "0")
        db = eng.upload(batch)
        dm = torch.zeros((Wd, batch.n), dtype=torch.int32, device="cuda:0")
        de = torch.zeros_like(dm)
        cm = torch.zeros_like(dm)
        flags = torch.ones(batch.n, dtype=torch.uint8, device="cuda:0")  # (stale flags must be cleared)
        hits = torch.zeros(len(rules), dtype=torch.int64, device="cuda:0")
        hc = torch.zeros_like(hits)
        for _ in range(3):  # the fused / streamed choice follows the previous evaluation
            db.eval_hits(dm.data_ptr(), de.data_ptr(), hits.data_ptr(), 0)
            db.eval_compact(cm.data_ptr(), flags.data_ptr(), hc.data_ptr(), 0)
        torch.cuda.synchronize()
        out.append([x.cpu().numpy() for x in (dm, de, hits, cm, flags, hc)])
        db.free()
    for o in out[:-1]:
        for a, b in zip(o, out[-1]):
            assert np.array_equal(a, b)
    assert out[0][2].sum() > 0 and out[0][1].any() and out[0][4].any()
    assert np.array_equal(out[0][0], out[0][3]) and np.array_equal(out[0][2], out[0][5])


def test_deferred_pairs_plain_c4(mxp, monkeypatch):
    """The bench's C4 family (no continuations, no errors) at 10k rules: against the oracle.  Value
    classes at their default threshold: the header columns (17 values) take them, the path column
    (a class per request) stays with the prefix index."""
    manifest, rules, batch = W.c4_workload(n_rules=10_000, n_requests=2048 + 7, seed=4)
    eng = engine_for(mxp, monkeypatch, {}, manifest, rules, flags="0")
    assert deferred_ran(eng, batch, len(rules))
    compare(eng, oracle.OracleEvaluator(manifest), rules, batch)


def test_deferred_pairs_windows_and_quad_overflow(mxp, monkeypatch):
    """17k rules (over 32 fill chunks: mxp_dtp_sort_kernel files them in two windows) led by 64
    copies of `request.path.startsWith("/w1")` (one canonical rule and 63 aliases in the first
    chunk: a matching request's quad holds far more than 8 pairs there -- the rest go through the
    overflow list).  Value classes at their default threshold (headers yes, paths no)."""
    manifest, rules, batch = W.c4_workload(n_rules=17_000, n_requests=4000 + 3, seed=49)
    rules = ['request.path.startsWith("/w1")'] * 64 + rules
    eng = engine_for(mxp, monkeypatch, {}, manifest, rules, flags="0")
    assert deferred_ran(eng, batch, len(rules))
    got, want = compare(eng, oracle.OracleEvaluator(manifest), rules, batch)
    assert (want[:, 0] == 1).sum() > 100


@pytest.mark.parametrize("env", PATHS, ids=["lists", "overflow", "rerun"])
def test_deferred_pairs_plain_fill_parity(mxp, monkeypatch, env):
    """Route rules matched on paths alone (no value classes): the indexed groups are plain fill
    chunks, written by mxp_fill_dtp_kernel with the pairs merged; continuations give error pairs."""
    manifest, rules, batch = W.c4_workload(n_rules=1500, n_requests=8000 + 13, seed=50, cont_frac=0.5,
                                           paths_only=True)
    eng = engine_for(mxp, monkeypatch, env, manifest, rules, flags="0")
    assert deferred_ran(eng, batch, len(rules))
    got, want = compare(eng, oracle.OracleEvaluator(manifest), rules, batch, sample_msgs=300)
    assert (want == 1).sum() > 1000 and (want >= 2).sum() > 50


def test_deferred_pairs_plain_fill_device_identical(mxp, monkeypatch):
    """Paths-only routes: device bitmaps, hit counters and compact output with deferred pairs on
    (through mxp_fill_dtp_kernel) equal deferred pairs off."""
    import torch
    manifest, rules, batch = W.c4_workload(n_rules=3000, n_requests=60_000 + 7, seed=51, cont_frac=0.2,
                                           paths_only=True)
    Wd = (len(rules) + 31) // 32
    out = []
    for env in ({}, {"MXP_DTP": "0"}):
        eng = engine_for(mxp, monkeypatch, env, manifest, rules, flags="0")
        assert deferred_ran(eng, batch, len(rules)) == (not env)
        db = eng.upload(batch)
        dm = torch.zeros((Wd, batch.n), dtype=torch.int32, device="cuda:0")
        de = torch.zeros_like(dm)
        cm = torch.zeros_like(dm)
        flags = torch.ones(batch.n, dtype=torch.uint8, device="cuda:0")  # (stale flags must be cleared)
        hits = torch.zeros(len(rules), dtype=torch.int64, device="cuda:0")
        hc = torch.zeros_like(hits)
        for _ in range(3):
            db.eval_hits(dm.data_ptr(), de.data_ptr(), hits.data_ptr(), 0)
            db.eval_compact(cm.data_ptr(), flags.data_ptr(), hc.data_ptr(), 0)
        torch.cuda.synchronize()
        out.append([x.cpu().numpy() for x in (dm, de, hits, cm, flags, hc)])
        db.free()
    for a, b in zip(out[0], out[1]):
        assert np.array_equal(a, b)
    assert out[0][2].sum() > 0 and out[0][1].any()


@pytest.mark.parametrize("env", PATHS[:2], ids=["lists", "overflow"])
def test_deferred_pairs_across_streams(mxp, monkeypatch, env):
    """Deferred launches queued back to back on two streams with no host synchronisation between
    them (two caller goroutines' streams): the second waits for the first's
    engine-wide pair scratch and overflow counters, so both batches' bitmaps equal those of the
    engine with deferred pairs off (MXP_DTP=0); then a bigger batch (the scratch grows) on the
    first stream."""
    import torch
    manifest, rules, big = W.c4_workload(n_rules=1200, n_requests=20000, seed=14)
    R = len(rules)
    Wd = (R + 31) // 32
    batches = [big.subset(np.arange(0, 9000)), big.subset(np.arange(9000, 17000)), big]

    def run(eng, streams):
        outs = []
        dbs = [eng.upload(b) for b in batches]
        bufs = []
        for db, b, s in zip(dbs, batches, streams):
            dm = torch.full((Wd, b.n), -1, dtype=torch.int32, device="cuda:0")
            de = torch.full_like(dm, -1)
            hits = torch.zeros(R, dtype=torch.int64, device="cuda:0")
            db.eval_hits(dm.data_ptr(), de.data_ptr(), hits.data_ptr(), s.cuda_stream)
            bufs.append((dm, de, hits))
        torch.cuda.synchronize()
        for dm, de, hits in bufs:
            outs.append((dm.cpu().numpy(), de.cpu().numpy(), hits.cpu().numpy()))
        for db in dbs:
            db.free()
        return outs
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    eng = engine_for(mxp, monkeypatch, env, manifest, rules)
    assert deferred_ran(eng, batches[0], R)
    got = run(eng, [s1, s2, s1])
    ref = run(engine_for(mxp, monkeypatch, {"MXP_DTP": "0"}, manifest, rules), [s1, s1, s1])
    for a, b in zip(got, ref):
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
    assert (got[2][0] != 0).any()


@pytest.mark.parametrize("chunks", ["2", "5"])
def test_deferred_pairs_request_chunks(mxp, monkeypatch, chunks):
    """The deferred-pair request chunks (MXP_DTP_CHUNKS: chunk c's index and sort kernels on the
    side stream beside chunk c - 1's fill; off by default, DESIGN §8 experiments): bitmaps and hit
    counters equal those of the unchunked engine, on C4 routes with index error pairs and on C2,
    over a ragged batch, three evaluations back to back."""
    import torch
    for wl in ("c4", "c2"):
        if wl == "c4":
            manifest, rules, batch = W.c4_workload(n_rules=1500, n_requests=12345, seed=21)
        else:
            manifest, rules, batch = W.c2_workload(n_rules=1500, n_requests=12345, seed=21)
        R = len(rules)
        Wd = (R + 31) // 32
        outs = []
        for env in ({"MXP_DTP_CHUNKS": chunks}, {}):
            monkeypatch.delenv("MXP_DTP_CHUNKS", raising=False)
            eng = engine_for(mxp, monkeypatch, env, manifest, rules)
            db = eng.upload(batch)
            dm = torch.full((Wd, batch.n), -1, dtype=torch.int32, device="cuda:0")
            de = torch.full_like(dm, -1)
            hits = torch.zeros(R, dtype=torch.int64, device="cuda:0")
            torch.cuda.synchronize()
            s = torch.cuda.Stream()
            for _ in range(3):
                db.eval_hits(dm.data_ptr(), de.data_ptr(), hits.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize()
            outs.append((dm.cpu().numpy(), de.cpu().numpy(), hits.cpu().numpy()))
            db.free()
        for x, y in zip(*outs):
            assert np.array_equal(x, y), wl
        assert outs[0][2].sum() > 0
