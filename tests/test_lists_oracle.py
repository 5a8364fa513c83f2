"""List-adapter restatement (oracle/lists.py + lists_oracle.c) against the reference's list tests
(mixer/adapter/list/list_test.go, transcribed into tests/golden/list_cases.json)."""
import json
import os

import numpy as np
import pytest

import lists as L

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "list_cases.json")))


def oracle_list(spec):
    if spec["type"] == L.REGEX:
        return L.RegexList(spec["entries"], spec["overrides"])
    if spec["type"] == L.IP_ADDRESSES:
        return L.IPList(spec["entries"], spec["overrides"])
    return L.StringList(spec["entries"], spec["overrides"], case_insensitive=spec["type"] == L.CASE_INSENSITIVE_STRINGS)


@pytest.mark.parametrize("spec", CASES["lists"], ids=lambda s: s["name"])
def test_reference_list_table(spec):
    if "parse_error" in spec:
        with pytest.raises(L.ListParseError) as ei:
            oracle_list(spec)
        assert str(ei.value) == spec["parse_error"]
        return
    lst = oracle_list(spec)
    syms = [c[0] for c in spec["cases"]]
    got = L.codes(lst.found(syms), spec["blacklist"])
    assert list(got) == [c[1] for c in spec["cases"]]


def test_ip_semantics_edges():
    lst = L.IPList(["10.0.0.0/8", "::1", "::ffff:1.2.3.0/120", "2001:db8::/32", "1.2.3.4/0"])
    # "::1" -> "::1/32" (IPv6 /32); v4-mapped IPv6 net acts as IPv4 1.2.3.0/24; /0 matches every IPv4
    syms = ["10.1.2.3", "::1", "0:0::5", "1.2.3.200", "2001:db8:ffff::1", "2001:db9::1", "8.8.8.8",
            "::ffff:10.0.0.1", "010.1.1.1", "1.2.3", "::ffff:8.8.8.8"]
    assert list(lst.found(syms)) == [1, 1, 1, 1, 1, 0, 1, 1, 1, -1, 1]


def test_to_upper_ascii():
    assert L.go_to_upper(b"AbC-z{") == b"ABC-Z{"


def test_regex_list_errors():
    with pytest.raises(L.ListParseError) as ei:
        L.RegexList(["a+", "(b"], [])
    assert str(ei.value) == "error parsing regexp: missing closing ): `(b`"


@pytest.mark.parametrize("ci", [False, True])
def test_c_string_list_equals_python(ci):
    """lists_oracle.c's string list (the compiled CPU baseline: hash set + Go strings.ToUpper in C)
    against the Python restatement: entry counts and membership, non-ASCII and invalid UTF-8
    included; its ToUpper against go_to_upper byte for byte."""
    import oracle
    from istio_amd import workloads as W
    entries, syms = W.ci_unicode_list(n_entries=2000, n_lookups=20000, seed=45)
    py, c = L.StringList(entries[:1500] + [""], entries[1500:], ci), L.CStringList(entries[:1500] + [""], entries[1500:], ci)
    assert py.num_entries() == c.num_entries()
    assert np.array_equal(py.found(syms), c.found(syms, threads=4))
    lib = oracle.lib()
    import ctypes
    for s in syms[:3000]:
        b = s.encode("utf-8", "surrogateescape")
        out = ctypes.create_string_buffer(3 * len(b) + 4)
        n = lib.oracle_go_to_upper(b, len(b), out)
        assert out.raw[:n] == L.go_to_upper(b), b
