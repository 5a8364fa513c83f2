"""The batch value model (istio_amd/bags.py) on its own: every Python bag value goes through
BagBatch.from_bags / from_columns into the columnar layout of include/mxp_batch.h and comes back
unchanged through BagBatch.get (attribute.Bag.Get), with the Go dynamic type the interpreter
type-asserts (interpreterRun.go:455-708).  The oracle and the engine both read this encoding, so a
fault here would be invisible to the parity tests; this pins it independently of both."""
import ctypes

import numpy as np
import pytest

from istio_amd import bags as B
from istio_amd import workloads as W


def _same(a, b):
    """Go-value equality including the dynamic type (GoInt64 vs GoDuration, str vs bytes, ...)."""
    norm = {int: B.GoInt64, float: B.GoFloat64}
    ta, tb = norm.get(type(a), type(a)), norm.get(type(b), type(b))
    if ta is not tb:
        return False
    if isinstance(a, float) and np.isnan(a):
        return np.isnan(b)
    if isinstance(a, float):
        return a == b and np.signbit(a) == np.signbit(b)
    return a == b


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fuzz_bags_round_trip(seed):
    bags = W.fuzz_bags(400, seed=seed)
    names = list(W.DEFAULT_TEST_MANIFEST) + ["not.in.any.bag"]
    batch = B.BagBatch.from_bags(bags, names=names)
    assert batch.n == len(bags)
    for q, bag in enumerate(bags):
        for name in names:
            got, found = batch.get(q, name)
            assert found == (name in bag), (q, name)
            if found:
                assert _same(bag[name], got), (q, name, bag[name], got)


def test_every_go_type_and_edge_value():
    vals = ["", "plain", "ünïcödé", "\udcff\udcferaw", B.GoInt64(-(1 << 63)), B.GoInt64((1 << 63) - 1), 7,
            B.GoFloat64(-0.0), B.GoFloat64(float("inf")), B.GoFloat64(float("nan")), 2.5, True, False,
            B.GoDuration(-1), B.GoDuration(10**18), B.GoTime(-62135596800, 0), B.GoTime(1420211075, 999_999_999),
            b"", bytes(range(256)), bytearray(b"\x00\x01"), {}, {"k": "v", "": "", "x": "ü"},
            B.GoOther("20"), B.GoOther("")]
    bags = [{"a": v} for v in vals] + [{}]
    batch = B.BagBatch.from_bags(bags, names=["a"])
    for q, v in enumerate(vals):
        got, found = batch.get(q, "a")
        assert found
        want = bytes(v) if isinstance(v, bytearray) else v
        assert _same(want, got), (v, got)
    assert batch.get(len(vals), "a") == (None, False)
    # kinds as mxp_batch.h numbers them
    assert [int(k) for k in batch.kinds[0][:6]] == [B.STRING] * 4 + [B.INT64] * 2


def test_duplicate_strings_share_or_not_ids_but_compare_by_bytes():
    bags = [{"a": "x", "b": "x"}, {"a": "x", "m": {"x": "x"}}]
    batch = B.BagBatch.from_bags(bags, names=["a", "b", "m"])
    assert batch.get(0, "a") == ("x", True) and batch.get(0, "b") == ("x", True)
    assert batch.get(1, "m") == ({"x": "x"}, True)


def test_from_columns_matches_from_bags():
    """The numpy column builder (the large synthetic workloads) against the dict builder."""
    manifest, rules, batch = W.c2_workload(n_rules=10, n_requests=500, seed=12)
    bags = [{nm: v for nm in batch.names for v, f in [batch.get(q, nm)] if f} for q in range(batch.n)]
    again = B.BagBatch.from_bags(bags, names=batch.names)
    for q in range(batch.n):
        for nm in batch.names:
            a, b = batch.get(q, nm), again.get(q, nm)
            assert a[1] == b[1] and (not a[1] or _same(a[0], b[0])), (q, nm, a, b)


def test_c_struct_layout_matches_the_header():
    """Field offsets of the ctypes mirror equal mxp_batch.h's struct on this ABI (x86-64 / LP64)."""
    batch = B.BagBatch.from_bags([{"a": "x", "t": B.GoTime(1, 2), "m": {"k": "v"}}], names=["a", "t", "m"])
    s = batch.c_struct()
    fields = [f[0] for f in type(s)._fields_]
    assert fields == ["n_requests", "n_columns", "column_names", "kinds", "values", "n_strings", "str_bytes",
                      "str_offsets", "n_times", "time_sec", "time_nsec", "n_maps", "map_offsets", "map_keys",
                      "map_values"]
    off = {f: getattr(type(s), f).offset for f in fields}
    assert off == {"n_requests": 0, "n_columns": 4, "column_names": 8, "kinds": 16, "values": 24, "n_strings": 32,
                   "str_bytes": 40, "str_offsets": 48, "n_times": 56, "time_sec": 64, "time_nsec": 72,
                   "n_maps": 80, "map_offsets": 88, "map_keys": 96, "map_values": 104}
    assert ctypes.sizeof(s) == 112
    assert s.n_requests == 1 and s.n_columns == 3 and s.n_times == 1 and s.n_maps == 1


def test_narrow_batch_layout():
    """bags.NarrowBatch (mxp_bag_batch2): id / BOOL columns travel as u32 (exact copies), numeric
    columns stay u64, offsets become u32; C2 batches cross the link in ~30-39 % fewer bytes."""
    import numpy as np
    from istio_amd.bags import BagBatch, NarrowBatch
    b = BagBatch.from_bags(W.fuzz_bags(300, seed=3, p_wrong=0.0), names=list(W.DEFAULT_TEST_MANIFEST))
    nb = NarrowBatch(b)
    for c, name in enumerate(b.names):
        numeric = bool(np.isin(b.kinds[c], (2, 3, 5)).any())
        assert bool(nb.narrow[c]) == (not numeric), name
        if nb.narrow[c]:
            assert np.array_equal(nb.values32[c].astype(np.uint64), b.values[c])
    assert np.array_equal(nb.str_offsets32.astype(np.uint64), b.str_offsets)
    cs = nb.c_struct()
    assert not cs.base.str_offsets and cs.str_offsets32 and cs.base.n_requests == 300
    _, _, c2 = W.c2_workload(n_rules=50, n_requests=1 << 16, seed=2)
    wide = sum(a.nbytes for a in list(c2.kinds) + list(c2.values) + [c2.str_blob, c2.str_offsets])
    assert NarrowBatch(c2).wire_bytes() < 0.72 * wide
