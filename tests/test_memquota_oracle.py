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
