"""String heads (kargs.heads, kernels.hip mxp_heads_kernel): every packed batch carries, per column
and request, a string value's first 12 bytes and its length, and the guard-index kernel hashes and
verifies prefix / composite keys of at most 12 bytes from them instead of the string's descriptor
and bytes.  Bar: bit-exact against the oracle, and against the engine without heads (MXP_HEADS=0),
at the boundaries the head format has -- key lengths 1..16 around the 8-byte word and the 12-byte
head, subjects shorter than, equal to and longer than the key and the head, the empty string,
non-ASCII bytes, absent and non-string values of the probed column."""
import numpy as np
import pytest

import oracle
from istio_amd.bags import BagBatch
from test_gpu_parity import compare, gpu_codes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mxp(libmxp):
    import istio_amd.engine as mxp
    return mxp


MANIFEST = {"request.path": "STRING", "destination.service": "STRING", "request.size": "INT64"}


SHORT = ["/", "/a", "/ab", "/abcdefg", "/abcdefgh", "/abcdefgh1", "/abcdefghij", "/abcdefghijk",
         "/été/x", "/abcdefghé", "/abcdefghi\u00e9"]
LONG = SHORT + ["/abcdefghijkl", "/abcdefghijklm", "/abcdefghijklmnop", "/" + "x" * 254, "/" + "x" * 299]
# (keys of 255 bytes and more: the composite entry stores min(length, 255) -- vm.h)


def head_rules(keys=SHORT):
    """keys of at most 12 bytes (the index reads heads) or some longer (it reads the strings)"""
    assert all(len(k.encode()) <= 12 for k in SHORT)
    rules = []
    for k in keys:
        rules.append('request.path.startsWith("%s")' % k)  # prefix index
        rules.append('destination.service == "s1" && request.path.startsWith("%s")' % k)  # composite
        rules.append('destination.service == "s2" && request.path.startsWith("%s") && request.size == 10' % k)
    return rules, keys


def head_bags(keys, n, seed):
    rng = np.random.default_rng(seed)
    subjects = [""] + keys + [k[:-1] for k in keys if len(k) > 1] + [k + "z" for k in keys] + \
        ["/abcdefghijklmnopqrstuvwxyz", "/abcdefghijkl/", "/abcdefghijké", "x/abcdefgh"]
    bags = []
    for i in range(n):
        b = {"destination.service": ["s1", "s2", "s3"][int(rng.integers(0, 3))], "request.size": int(rng.integers(0, 20))}
        r = rng.random()
        if r < 0.05:
            pass  # request.path absent
        else:
            b["request.path"] = subjects[int(rng.integers(0, len(subjects)))]
        if rng.random() < 0.03:
            del b["destination.service"]
        bags.append(b)
    return BagBatch.from_bags(bags)


@pytest.mark.parametrize("heads", ["1", "0"])
@pytest.mark.parametrize("keyset", ["short", "long"])
def test_heads_prefix_parity(mxp, monkeypatch, heads, keyset):
    monkeypatch.setenv("MXP_HEADS", heads)
    rules, keys = head_rules(SHORT if keyset == "short" else LONG)
    batch = head_bags(keys, 3000, seed=11)
    eng = mxp.Engine(0)
    eng.set_vocabulary(MANIFEST)
    st = eng.compile(rules)
    assert (st == 0).all(), st
    compare(eng, oracle.OracleEvaluator(MANIFEST), rules, batch)


def test_heads_on_off_identical_c2(mxp, monkeypatch):
    """The benched C2 family (composite keys of 10 and 11 bytes: read from heads) at 64k requests:
    the same match bits and error flags with and without heads."""
    from istio_amd import workloads as W
    manifest, rules, batch = W.c2_workload(n_rules=2000, n_requests=65536, seed=5)
    got = {}
    for h in ("1", "0"):
        monkeypatch.setenv("MXP_HEADS", h)
        eng = mxp.Engine(0)
        eng.set_vocabulary(manifest)
        assert (eng.compile(rules) == 0).all()
        got[h] = gpu_codes(eng, batch)
    assert np.array_equal(got["1"], got["0"])
