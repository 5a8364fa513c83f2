"""memquota restatement (oracle/memquota.py) against the reference's own tables
(memquota_test.go TestAllocAndRelease, rollingWindow_test.go TestAlloc / TestRelease,
transcribed into tests/golden/memquota_cases.json)."""
import json
import os

import memquota as M

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "memquota_cases.json")))
BASE_NS = 1_500_000_000 * 10**9  # "now" of the table; only differences matter


def test_window_alloc_table():
    t = CASES["window_alloc"]
    w = M.RollingWindow(t["limit"], t["ticks"])
    for amount, tick, avail, result in t["cases"]:
        assert w.alloc(amount, tick) is result
        assert w.avail == avail


def test_window_release_table():
    t = CASES["window_release"]
    w = M.RollingWindow(t["limit"], t["ticks"])
    for aa, at, ra, rt, rr, avail in t["cases"]:
        assert w.alloc(aa, at)
        assert w.release(ra, rt) == rr
        assert w.avail == avail


def test_alloc_and_release_table():
    t = CASES["alloc_and_release"]
    mq = M.Memquota({k: tuple(v) for k, v in t["limits"].items()})
    dd = M.Dedup()
    for name, dedup, aa, ar, abe, exp, sec, ra, rr in t["cases"]:
        now = BASE_NS + sec * 10**9
        if aa != 0:
            got = dd("A" + dedup, lambda: mq.handle(name, aa, abe, now))
        else:
            got = 0
        assert got == ar
        if ra != 0:
            got = dd("R" + dedup, lambda: mq.handle(name, -ra, False, now))
        else:
            got = 0
        assert got == rr


def test_c_restatement_matches_python():
    """memquota_oracle.c (the bench's CPU baseline, keys in parallel) against the Python
    restatement on random batches: cells and windows, best effort, frees past what is in use,
    frees of absent keys, out-of-range keys, time moving across window slots."""
    import numpy as np
    rng = np.random.default_rng(5)
    K = 40
    mx = rng.integers(1, 200, size=K)
    vd = np.where(rng.random(K) < 0.5, 0, rng.integers(1, 4, size=K) * 10**9)
    py = M.Memquota({k: (int(mx[k]), int(vd[k])) for k in range(K)})
    c = M.CMemquota(mx, vd)
    now = BASE_NS
    for batch in range(12):
        n = 3000
        keys = rng.integers(-2, K + 2, size=n).astype(np.int32)
        amounts = rng.integers(-60, 80, size=n)
        be = rng.random(n) < 0.4
        got = c.handle_batch(keys, amounts, be, now, threads=4)
        want = [py.handle(int(k), int(a), bool(b), now) if 0 <= k < K else 0 for k, a, b in zip(keys, amounts, be)]
        assert got.tolist() == want, batch
        now += int(rng.integers(0, 7)) * 10**8
