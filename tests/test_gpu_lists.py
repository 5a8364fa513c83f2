"""GPU list adapter (mxp_list_create / mxp_list_check) against the list restatement
(oracle/lists.py): the reference's list tests, then C3-shaped CIDR and string lists (smaller than
BASELINE configs[2]: the oracle's IP check is the reference's linear scan).  Bar: identical status
codes per symbol, identical parse errors and entry counts."""
import json
import os

import numpy as np
import pytest

import lists as L
from istio_amd import workloads as W

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "list_cases.json")))


@pytest.fixture(scope="module")
def eng(libmxp):
    import istio_amd.engine as mxp
    return mxp.Engine(0)


@pytest.mark.parametrize("spec", CASES["lists"], ids=lambda s: s["name"])
def test_reference_list_table_on_gpu(eng, spec):
    from istio_amd.engine import MxpError
    if "parse_error" in spec:
        with pytest.raises(MxpError) as ei:
            eng.list_create(spec["type"], spec["entries"], spec["overrides"])
        assert str(ei.value).endswith(spec["parse_error"])
        return
    lst = eng.list_create(spec["type"], spec["entries"], spec["overrides"])
    got = lst.check([c[0] for c in spec["cases"]], spec["blacklist"])
    assert list(got) == [c[1] for c in spec["cases"]]


@pytest.mark.parametrize("blacklist", [False, True])
def test_c3_ip_list_parity(eng, blacklist):
    entries, syms = W.c3_ip_list(n_entries=3000, n_lookups=40000, seed=31)
    lst = eng.list_create(L.IP_ADDRESSES, entries, ["11.11.11.11", "bad-override"])
    ref = L.IPList(entries, ["11.11.11.11", "bad-override"])
    assert lst.num_entries() == ref.num_entries()
    want = L.codes(ref.found(syms, threads=16), blacklist)
    got = lst.check(syms, blacklist)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(syms[i], int(got[i]), int(want[i])) for i in bad[:5]]
    assert set(np.unique(want)) >= ({0, 3, 7} if blacklist else {0, 3, 5})


@pytest.mark.parametrize("kind", [L.STRINGS, L.CASE_INSENSITIVE_STRINGS])
def test_c3_string_list_parity(eng, kind):
    entries, syms = W.c3_string_list(n_entries=20000, n_lookups=100000, seed=32)
    lines = entries[:15000] + [""]  # an empty line: skipped
    lst = eng.list_create(kind, lines, entries[15000:])
    ref = L.StringList(lines, entries[15000:], case_insensitive=kind == L.CASE_INSENSITIVE_STRINGS)
    assert lst.num_entries() == ref.num_entries()
    want = L.codes(ref.found(syms), False)
    got = lst.check(syms)
    assert np.array_equal(got, want)
    assert (want == 0).sum() > 1000 and (want == 5).sum() > 1000


def test_c3_regex_list_parity(eng):
    pats, syms = W.c3_regex_list(n_patterns=200, n_lookups=1500, seed=33)
    lst = eng.list_create(L.REGEX, pats[:150] + [""], pats[150:])
    ref = L.RegexList(pats[:150] + [""], pats[150:])
    assert lst.num_entries() == ref.num_entries() == 200
    want = L.codes(ref.found(syms), False)
    got = lst.check(syms)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(syms[i], int(got[i]), int(want[i])) for i in bad[:5]]
    assert (want == 0).sum() > 300 and (want == 5).sum() > 300


def test_regex_list_compile_error(eng):
    from istio_amd.engine import MxpError
    with pytest.raises(MxpError) as ei:
        eng.list_create(L.REGEX, ["a+", "(b"], [])
    assert str(ei.value).endswith("error parsing regexp: missing closing ): `(b`")
