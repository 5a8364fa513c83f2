"""Malformed columnar batches are rejected at the boundary (engine.cpp check_batch), before any packer
or host pass reads them: ids past their tables, offsets running backwards, unknown kinds.  The
reference answers an undefined dictionary index with an error, not a crash
(mixer/pkg/attribute/protoBag.go:255-265); SURVEY.md §5 asks the same of a device error.

CPU: mxp_batch_pack_host on a host-only engine (the host packer would index with the bad ids).
GPU: mxp_batch_upload and mxp_eval_batch get MXP_ERR_ARG for each malformed batch, and the same
engine then evaluates a good batch bit-exact against the oracle."""
import numpy as np
import pytest

from istio_amd import workloads as W
from istio_amd.bags import BagBatch, GoTime

MANIFEST = dict(W.DEFAULT_TEST_MANIFEST)
RULES = [
    'as == "x"',
    'ar["k"] == "v"',
    'at == timestamp("2017-01-01T00:00:00Z")',
    'aip == ip("10.0.0.1")',
    'bs.startsWith("a") || ai == 3',
    'match(as, "x*")',
]


def good_batch(n=300):
    rng = np.random.default_rng(7)
    bags = []
    for q in range(n):
        b = {"as": rng.choice(["x", "y", "xa"]), "ai": int(rng.integers(0, 5)), "bs": rng.choice(["ab", "b"]),
             "ar": {"k": rng.choice(["v", "w"]), "z": "1"},
             "at": GoTime(1483228800 + int(rng.integers(0, 2)), 0),
             "aip": bytes([10, 0, 0, int(rng.integers(0, 3))])}
        if q % 7 == 0:
            del b["ar"]
        bags.append(b)
    return BagBatch.from_bags(bags, names=list(MANIFEST))


def clone(b):
    return BagBatch(b.n, b.names, [k.copy() for k in b.kinds], [v.copy() for v in b.values], b.str_blob.copy(),
                    b.str_offsets.copy(), b.time_sec.copy(), b.time_nsec.copy(), b.map_offsets.copy(),
                    b.map_keys.copy(), b.map_values.copy())


def _col(b, name):
    return b.names.index(name)


def malformed(b):
    """(label, expected message fragment, batch) for each malformed variant of `b`."""
    out = []

    def variant(label, frag, f):
        x = clone(b)
        f(x)
        out.append((label, frag, x))

    def set_val(name, v):
        def f(x):
            x.values[_col(x, name)] = x.values[_col(x, name)].copy()
            x.values[_col(x, name)][5] = v
        return f

    ns = b.n_strings
    variant("string id", "'as' request 5: id", set_val("as", ns))
    variant("bytes id", "'aip' request 5: id", set_val("aip", ns + 9))
    variant("time id", ">= n_times", set_val("at", len(b.time_sec)))
    variant("map id", ">= n_maps", set_val("ar", 1 << 40))

    def kind(x):
        x.kinds[_col(x, "bs")] = x.kinds[_col(x, "bs")].copy()
        x.kinds[_col(x, "bs")][9] = 10
    variant("kind", "kind 10 > MXP_OTHER", kind)

    def soff(x):
        x.str_offsets = x.str_offsets.copy()
        x.str_offsets[3], x.str_offsets[4] = x.str_offsets[4] + 100, x.str_offsets[3]
    variant("string offsets", "str_offsets[", soff)

    def moff(x):
        x.map_offsets = x.map_offsets.copy()
        x.map_offsets[2] = x.map_offsets[3] + 1
    variant("map offsets", "map_offsets[", moff)

    def mkey(x):
        x.map_keys = x.map_keys.copy()
        x.map_keys[1] = ns + 1
    variant("map key", "key id", mkey)

    def mval(x):
        x.map_values = x.map_values.copy()
        x.map_values[4] = 1 << 31
    variant("map value", "value id", mval)
    return out


@pytest.fixture(scope="module")
def mxp(libmxp):
    import istio_amd.engine as mxp
    return mxp


def test_check_batch_host(mxp):
    eng = mxp.Engine(-1)
    eng.set_vocabulary(MANIFEST)
    assert (eng.compile(RULES) == 0).all()
    b = good_batch()
    eng.pack_host(b)  # the good batch packs
    bad = malformed(b)
    assert len(bad) == 9
    for label, frag, x in bad:
        with pytest.raises(mxp.MxpError) as ei:
            eng.pack_host(x)
        msg = str(ei.value)
        assert "failed (1)" in msg and "malformed batch" in msg and frag in msg, (label, msg)
    eng.pack_host(b)  # and still does afterwards


def test_check_batch_unread_columns_ignored(mxp):
    """Columns no rule reads are never read, so they are not checked either."""
    eng = mxp.Engine(-1)
    eng.set_vocabulary(MANIFEST)
    assert (eng.compile(['as == "x"']) == 0).all()
    b = good_batch()
    x = clone(b)
    x.values[_col(x, "bs")] = x.values[_col(x, "bs")].copy()
    x.values[_col(x, "bs")][3] = 1 << 50
    eng.pack_host(x)


@pytest.mark.gpu
def test_check_batch_device_then_good_batch(mxp):
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import oracle
    eng = mxp.Engine(0)
    eng.set_vocabulary(MANIFEST)
    assert (eng.compile(RULES) == 0).all()
    b = good_batch()
    for label, frag, x in malformed(b):
        with pytest.raises(mxp.MxpError) as ei:
            eng.upload(x)
        assert "failed (1)" in str(ei.value) and frag in str(ei.value), label
        with pytest.raises(mxp.MxpError) as ei:
            eng.eval_batch(x)
        assert "failed (1)" in str(ei.value) and frag in str(ei.value), label
    m, e = eng.eval_batch(b)
    got = mxp.bits_to_codes(m, e, len(RULES))
    want = oracle.oracle_matrix(oracle.OracleEvaluator(MANIFEST), RULES, b, threads=4)
    want = np.where(want >= 2, 2, want)
    assert np.array_equal(got, want)
    db = eng.upload(b)  # and the device batch path still works on the same engine
    db.free()
