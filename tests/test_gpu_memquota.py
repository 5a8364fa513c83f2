"""GPU batched memquota (mxp_quota_alloc) against the restatement (oracle/memquota.py): the
reference's TestAllocAndRelease table, then random batches (cells and 1 s / 60 s windows, allocs,
frees, best effort, advancing time) replayed in arrival order.  Bar: identical granted amounts."""
import json
import os

import numpy as np
import pytest

import memquota as M
from istio_amd import workloads as W

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "memquota_cases.json")))
BASE_NS = 1_500_000_000 * 10**9


@pytest.fixture(scope="module")
def eng(libmxp):
    import istio_amd.engine as mxp
    return mxp.Engine(0)


def test_reference_alloc_and_release_on_gpu(eng):
    t = CASES["alloc_and_release"]
    names = list(t["limits"])
    q = eng.quota_create([t["limits"][n][0] for n in names], [t["limits"][n][1] for n in names])
    dd = M.Dedup()  # DeduplicationID stays with the caller (the Go shim)
    for name, dedup, aa, ar, abe, exp, sec, ra, rr in t["cases"]:
        now = BASE_NS + sec * 10**9
        k = names.index(name)
        got = dd("A" + dedup, lambda: int(q.alloc([k], [aa], [abe], now)[0])) if aa else 0
        assert got == ar
        got = dd("R" + dedup, lambda: int(q.alloc([k], [-ra], [0], now)[0])) if ra else 0
        assert got == rr


@pytest.mark.parametrize("radix", ["0", "1"])
def test_random_batches_parity(eng, monkeypatch, radix):
    """Bucketed by the counting sort (default up to 4095 keys) and by the radix sort (MXP_QUOTA_RADIX=1,
    the path for more keys)."""
    monkeypatch.setenv("MXP_QUOTA_RADIX", radix)
    mx, vd, keys, amounts, be = W.quota_workload(n_keys=200, n_requests=60000, seed=51)
    q = eng.quota_create(mx, vd)
    ref = M.Memquota({k: (int(mx[k]), int(vd[k])) for k in range(200)})
    now = BASE_NS
    for b in range(6):
        sl = slice(b * 10000, (b + 1) * 10000)
        got = q.alloc(keys[sl], amounts[sl], be[sl], now)
        want = np.array([ref.handle(int(k), int(a), bool(e), now) for k, a, e in zip(keys[sl], amounts[sl], be[sl])])
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (b, bad[:5], got[bad[:5]], want[bad[:5]])
        now += [50_000_000, 400_000_000, 3 * 10**9, 0, 61 * 10**9, 10**8][b]
    assert (want == 0).any() and (want > 0).any()


def test_device_out_of_range_keys_granted_zero(eng):
    """Device key ids >= n_keys (no host range check on the device path): granted 0, no state touched,
    the in-range requests unchanged -- including ids whose low bits alias a valid key."""
    import torch
    K = 100
    mx, vd, keys, amounts, be = W.quota_workload(n_keys=K, n_requests=5000, seed=53)
    bad = np.zeros(len(keys), dtype=bool)
    bad[::7] = True
    keys_dev = keys.copy()
    keys_dev[bad] = np.where(np.arange(bad.sum()) % 2, K + 28, 0xFFFFFFF0)  # 128 aliases key 0 at 7 bits
    q = eng.quota_create(mx, vd)
    dk = torch.from_numpy(keys_dev.view(np.int32).copy()).cuda()
    da = torch.from_numpy(amounts.copy()).cuda()
    db = torch.from_numpy(be.copy()).cuda()
    dg = torch.full((len(keys),), 99, dtype=torch.int64, device="cuda")
    delta = torch.zeros(K, dtype=torch.int64, device="cuda")
    q.alloc_device(len(keys), dk.data_ptr(), da.data_ptr(), db.data_ptr(), BASE_NS, 0, dg.data_ptr(), delta.data_ptr())
    torch.cuda.synchronize()
    got = dg.cpu().numpy()
    ref = M.Memquota({k: (int(mx[k]), int(vd[k])) for k in range(K)})
    want = np.array([0 if b else ref.handle(int(k), int(a), bool(e), BASE_NS)
                     for k, a, e, b in zip(keys, amounts, be, bad)])
    assert np.array_equal(got, want)
    want_delta = np.zeros(K, dtype=np.int64)
    np.add.at(want_delta, keys[~bad].astype(np.int64), (np.sign(amounts) * want)[~bad])  # allocs - frees
    assert np.array_equal(delta.cpu().numpy(), want_delta)


def test_release_across_many_window_slots(eng):
    """A 60 s window (600 slots) filled one tick at a time, then frees that walk back over more than
    64 slots at once (the kernel releases 64 slots per step with a prefix sum over the lanes),
    including frees larger than everything held; two keys so the workgroup has a second wave."""
    mx = [100_000, 100_000]
    vd = [60 * 10**9, 60 * 10**9]
    q = eng.quota_create(mx, vd)
    ref = M.Memquota({k: (mx[k], vd[k]) for k in range(2)})
    rng = np.random.default_rng(7)
    now = BASE_NS
    for step in range(260):  # one batch per tick (100 ms): allocations land in distinct slots
        keys = np.array([0, 1, 0, 1], dtype=np.uint32)
        amounts = rng.integers(1, 5, size=4).astype(np.int64)
        if step in (150, 200, 259):  # frees spanning many slots, then one larger than all held
            amounts = np.array([-70, -90, -400, -5000], dtype=np.int64)
        be = np.zeros(4, dtype=np.uint8)
        got = q.alloc(keys, amounts, be, now)
        want = np.array([ref.handle(int(k), int(a), bool(e), now) for k, a, e in zip(keys, amounts, be)])
        assert np.array_equal(got, want), (step, got, want)
        now += 100_000_000


def test_replay_paths_parity(eng):
    """The kernel's three replays of a chunk -- 32-bit run steps (limits and in-use below 2^28,
    amounts below 2^20), 64-bit run steps, request-by-request for amounts past 2^55 or limits past
    2^61 -- and keys moving between them chunk to chunk: limits 0, small, 2^30, 2^62, a cell with a
    negative limit (best effort grants the negative room, a free takes it back); mid (2^20..2^24)
    and huge (2^56) amounts mixed into some batches; cells and windows."""
    rng = np.random.default_rng(61)
    mx = [0, 50, 5000, 5000, 1 << 30, 1 << 30, 1 << 62, 1 << 62, -7, 300, 3371, 1 << 27]
    vd = [0, 10**9, 0, 60 * 10**9, 0, 10**9, 0, 60 * 10**9, 0, 10**9, 60 * 10**9, 0]
    K = len(mx)
    q = eng.quota_create(mx, vd)
    ref = M.Memquota({k: (mx[k], vd[k]) for k in range(K)})
    now = BASE_NS
    for b in range(8):
        n = 3000
        keys = rng.choice(K, size=n, p=np.array([1, 1, 3, 3, 2, 2, 1, 1, 1, 2, 4, 1]) / 22).astype(np.uint32)
        amounts = rng.integers(1, 21, size=n).astype(np.int64)
        if b in (2, 3, 6):
            mid = rng.random(n) < 0.05
            amounts[mid] = rng.integers(1 << 20, 1 << 24, size=int(mid.sum()))
        if b in (4, 6):
            big = (rng.random(n) < 0.01) & np.isin(keys, [6, 7])
            amounts[big] = 1 << 56
        r = rng.random(n)
        amounts = np.where(r < 0.15, -amounts, amounts)
        amounts = np.where(r > 0.97, 0, amounts)
        be = (rng.random(n) < 0.5).astype(np.uint8)
        got = q.alloc(keys, amounts, be, now)
        want = np.array([ref.handle(int(k), int(a), bool(e), now) for k, a, e in zip(keys, amounts, be)])
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (b, [(int(keys[i]), int(amounts[i]), int(got[i]), int(want[i])) for i in bad[:5]])
        now += [50_000_000, 400_000_000, 3 * 10**9, 0, 61 * 10**9, 10**8, 0, 2 * 10**9][b]


def test_long_keys_in_pieces(eng):
    """Keys long enough to be cut into pieces (kPiece = 4096 requests, quota.hip): saturating keys
    (sync points within a few hundred requests), a key whose limit is never reached (no sync point:
    the first piece's wave replays it all), limit 0 (in sync from the first request), windows and
    cells, a long key with one amount past 2^55 (never cut), advancing time between batches; the
    per-key deltas against the oracle's grants."""
    import torch
    rng = np.random.default_rng(71)
    mx = [3371, 4035, 10**15, 0, 162, 2000, 1 << 40, 50]
    vd = [60 * 10**9, 0, 0, 10**9, 10**9, 0, 0, 60 * 10**9]
    K = len(mx)
    q = eng.quota_create(mx, vd)
    ref = M.Memquota({k: (mx[k], vd[k]) for k in range(K)})
    now = BASE_NS
    for b in range(4):
        n = 60000
        keys = rng.choice(K, size=n, p=np.array([6, 5, 3, 2, 3, 3, 2, 1]) / 25).astype(np.uint32)
        amounts = rng.integers(1, 21, size=n).astype(np.int64)
        r = rng.random(n)
        amounts = np.where(r < 0.1, -amounts, amounts)
        amounts = np.where(r > 0.98, 0, amounts)
        if b == 2:
            amounts[np.nonzero(keys == 6)[0][100]] = (1 << 56) + 5
        be = (rng.random(n) < 0.5).astype(np.uint8)
        dk = torch.from_numpy(keys.view(np.int32).copy()).cuda()
        da = torch.from_numpy(amounts.copy()).cuda()
        db = torch.from_numpy(be.copy()).cuda()
        dg = torch.zeros(n, dtype=torch.int64, device="cuda")
        delta = torch.zeros(K, dtype=torch.int64, device="cuda")
        q.alloc_device(n, dk.data_ptr(), da.data_ptr(), db.data_ptr(), now, 0, dg.data_ptr(), delta.data_ptr())
        torch.cuda.synchronize()
        got = dg.cpu().numpy()
        want = np.array([ref.handle(int(k), int(a), bool(e), now) for k, a, e in zip(keys, amounts, be)])
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (b, [(i, int(keys[i]), int(amounts[i]), int(got[i]), int(want[i])) for i in bad[:5]])
        want_delta = np.zeros(K, dtype=np.int64)
        np.add.at(want_delta, keys.astype(np.int64), np.sign(amounts) * want)
        assert np.array_equal(delta.cpu().numpy(), want_delta), b
        now += [400_000_000, 61 * 10**9, 0, 10**8][b]


def test_many_keys_radix_path(eng):
    """5000 keys (past the counting sort's 4095): the radix-sorted path, with long keys in pieces."""
    mx, vd, keys, amounts, be = W.quota_workload(n_keys=5000, n_requests=200_000, seed=57)
    q = eng.quota_create(mx, vd)
    ref = M.Memquota({k: (int(mx[k]), int(vd[k])) for k in range(5000)})
    got = q.alloc(keys, amounts, be, BASE_NS)
    want = np.array([ref.handle(int(k), int(a), bool(e), BASE_NS)
                     for k, a, e in zip(keys.tolist(), amounts.tolist(), be.tolist())])
    assert np.array_equal(got, want)


def test_bench_workload_against_oracle(eng):
    """The C5 batch bench.py times (1024 keys, 1,048,576 Zipf requests: the head key ~160k requests,
    cut into ~40 pieces), twice in a row (the second on the state the first left), against the oracle."""
    mx, vd, keys, amounts, be = W.quota_workload(n_keys=1024, n_requests=1 << 20, seed=5)
    q = eng.quota_create(mx, vd)
    ref = M.Memquota({k: (int(mx[k]), int(vd[k])) for k in range(1024)})
    now = BASE_NS
    for b in range(2):
        got = q.alloc(keys, amounts, be, now)
        want = np.array([ref.handle(int(k), int(a), bool(e), now)
                         for k, a, e in zip(keys.tolist(), amounts.tolist(), be.tolist())])
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (b, [(i, int(keys[i]), int(amounts[i]), int(got[i]), int(want[i])) for i in bad[:5]])
        now += 300_000_000
