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


def test_ip_symbol_edges(eng):
    """net.ParseIP edge symbols through both device parsers -- the register path for symbols of <= 15
    bytes whose first separator is '.', the byte path for the rest -- against the restatement:
    leading zeros, octets past 255, digit runs past Go's dtoi bound, missing / extra / empty parts,
    trailing garbage, 15 / 16 / 17-byte quads, v4-mapped and plain IPv6, spaces, empties."""
    entries = ["10.0.0.0/8", "1.2.3.4", "255.255.255.0/24", "0.0.0.0/32", "2001:db8::/32", "::ffff:7.7.7.0/120"]
    quads = ["1.2.3.4", "01.002.0003.4", "010.000.000.001", "10.1.2.3", "255.255.255.255", "255.255.255.2555",
             "0255.255.255.255", "256.1.1.1", "1.2.3", "1.2.3.4.5", "1..2.3", "1.2.3.", ".1.2.3", "1.2.3.4:80",
             "1.2.3.4 ", " 1.2.3.4", "99999999.1.1.1", "16777215.1.1.1", "0000000000001.2", "0.0.0.0", "00.0.0.0",
             "7.7.7.7", "::ffff:7.7.7.7", "::ffff:1.2.3.4", "2001:db8::1", "2001:db9::1", "::", "1.2.3.4/32",
             "", ".", ":", "1", "a.b.c.d", "1.2.3.-4", "1.2.3.+4", "1.2.3.4\x00", "10.255.255.255", "11.0.0.0",
             "10.0.0.0", "9.255.255.255", "255.255.255.1", "255.255.254.255", "1.2.3.4.", "0x1.2.3.4"]
    lst = eng.list_create(L.IP_ADDRESSES, entries, [])
    ref = L.IPList(entries, [])
    for blacklist in (False, True):
        want = L.codes(ref.found(quads, threads=1), blacklist)
        got = lst.check(quads, blacklist)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, [(quads[i], int(got[i]), int(want[i])) for i in bad[:8]]
    assert (want == 3).sum() > 10 and (want == 7).sum() > 5


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


@pytest.mark.parametrize("kind", [L.STRINGS, L.CASE_INSENSITIVE_STRINGS])
def test_string_symbol_lengths(eng, kind):
    """Symbols of 0..80 bytes at every alignment -- around the register path's 64-byte bound and the
    8-byte word edges -- hits, near misses (last byte changed) and case changes, ASCII and not,
    against the restatement."""
    rng = np.random.default_rng(41)
    alpha = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789-_./"
    entries = ["".join(rng.choice(list(alpha), size=k)) for k in range(1, 81) for _ in range(3)]
    entries += ["\u00e9t\u00e9-%d" % k for k in range(5)] + ["x" * 64, "y" * 65, "Z" * 63]
    syms = []
    for e in entries:
        syms += [e, e.swapcase(), e[:-1] + ("#" if e[-1] != "#" else "%"), e + "q", e[:-1]]
    syms += ["", "x" * 64, "X" * 64, "y" * 65, "z" * 63]
    for pad in range(8):  # every alignment of the symbols in the blob: a pad symbol first
        ss = ["p" * pad] + syms
        lst = eng.list_create(kind, entries, [])
        ref = L.StringList(entries, [], case_insensitive=kind == L.CASE_INSENSITIVE_STRINGS)
        want = L.codes(ref.found(ss), False)
        got = lst.check(ss)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, [(ss[i], int(got[i]), int(want[i])) for i in bad[:5]]


def test_regex_list_u16_parts_agree(eng, monkeypatch):
    """Regex lists as sorted u16 parts with depth-first state numbering (default) against u32 parts in
    the caller's order (MXP_LIST_RX16=0), with and without LDS staging, and against the restatement
    on a sample: identical codes."""
    pats, syms = W.c3_regex_list(n_patterns=4000, n_lookups=60000, seed=45)
    monkeypatch.setenv("MXP_LIST_RXP", "0")  # (the union parts: no literal-prefix dispatch)
    got = {}
    for rx16 in ("1", "0"):
        for lds in ("1", "0"):
            monkeypatch.setenv("MXP_LIST_RX16", rx16)
            monkeypatch.setenv("MXP_LIST_LDS", lds)
            lst = eng.list_create(L.REGEX, pats, [])
            got[(rx16, lds)] = lst.check(syms)
    ref = got[("1", "1")]
    for k, v in got.items():
        assert np.array_equal(v, ref), k
    sample = syms[:3000]
    want = L.codes(L.RegexList(pats, []).found(sample), False)
    assert np.array_equal(ref[:3000], want)


@pytest.mark.parametrize("kind", ["ip", "str"])
def test_list_paths_agree(eng, monkeypatch, kind):
    """The list kernels' paths give identical codes: IP family regrouping on / off, the register
    parse, the /16 directory and the string register path each off (MXP_LIST_OPT bits)."""
    if kind == "ip":
        entries, syms = W.c3_ip_list(n_entries=5000, n_lookups=60000, seed=43)
        lst = eng.list_create(L.IP_ADDRESSES, entries, [])
        settings = [("1", "255"), ("0", "255"), ("1", "0"), ("1", "1"), ("1", "2")]
    else:
        entries, syms = W.c3_string_list(n_entries=5000, n_lookups=60000, seed=44)
        lst = eng.list_create(L.CASE_INSENSITIVE_STRINGS, entries, [])
        settings = [("1", "255"), ("1", "0")]
    ref = None
    for split, opt in settings:
        monkeypatch.setenv("MXP_LIST_IP_SPLIT", split)
        monkeypatch.setenv("MXP_LIST_OPT", opt)
        got = lst.check(syms, True)
        if ref is None:
            ref = got
        assert np.array_equal(got, ref), (split, opt)


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


@pytest.mark.parametrize("case", ["small", "c3-10k", "nfa-parts", "multi-part"])
def test_regex_list_lds_staging(monkeypatch, case):
    """mxp_list_rx_kernel (the parts' hot DFA rows staged in LDS) against the global-memory walk
    (MXP_LIST_LDS=0, mxp_list_kernel) and the oracle: a 200-pattern list, the 10k-pattern C3 union
    staged in part (its DFA is far larger than the LDS budget), NFA parts between staged DFAs,
    and several union parts; ragged lookup counts past one grid-stride round (512 x 1024 lanes)."""
    import istio_amd.engine as mxp
    rng = np.random.default_rng(71)
    if case == "small":
        pats, syms = W.c3_regex_list(n_patterns=200, n_lookups=20_011, seed=72)
    elif case == "c3-10k":
        pats, syms = W.c3_regex_list(n_patterns=10_000, n_lookups=600_037, seed=73)
    elif case == "nfa-parts":
        from test_regex_product import NFA_PATTERNS, _nfa_subjects
        pats = ["^zz", NFA_PATTERNS[0], "x{3}", NFA_PATTERNS[2], "^é", "(?i)ab+c$"]
        syms = _nfa_subjects(rng, 5003) + ["zzz", "éa", "xxx", "ABBC", "abc", ""]
    else:
        pats, syms = W.c3_regex_list(n_patterns=50_000, n_lookups=80_021, seed=74)
    out = {}
    monkeypatch.setenv("MXP_LIST_RXP", "0")  # (the union parts: no literal-prefix dispatch)
    for lds in ("1", "0"):
        monkeypatch.setenv("MXP_LIST_LDS", lds)
        eng = mxp.Engine(0)
        lst = eng.list_create(L.REGEX, pats, [])
        out[lds] = (lst.check(syms), lst.check(syms, True))
    assert np.array_equal(out["1"][0], out["0"][0]) and np.array_equal(out["1"][1], out["0"][1])
    sample = rng.choice(len(syms), min(len(syms), 800), replace=False)
    want = L.codes(L.RegexList(pats).found([syms[i] for i in sample], threads=16), False)
    assert np.array_equal(out["1"][0][sample], want)
    assert (want == 0).sum() > 20 and (want == 5).sum() > 20


def test_regex_list_compile_error(eng):
    from istio_amd.engine import MxpError
    with pytest.raises(MxpError) as ei:
        eng.list_create(L.REGEX, ["a+", "(b"], [])
    assert str(ei.value).endswith("error parsing regexp: missing closing ): `(b`")


def _listentry_bags(n, seed):
    """Bags for listentry instances: source.labels with / without `version`, maps missing, paths,
    forwarded-for addresses (valid, invalid, absent)."""
    from istio_amd.bags import BagBatch
    rng = np.random.default_rng(seed)
    versions = ["v1", "v2", "v3", "V1", "", "canary"]
    bags = []
    for i in range(n):
        b = {}
        r = rng.random()
        if r < 0.8:
            labels = {"app": "ratings"}
            if rng.random() < 0.85:
                labels["version"] = versions[int(rng.integers(0, len(versions)))]
            b["source.labels"] = labels
        elif r < 0.9:
            b["source.labels"] = "not-a-map"
        if rng.random() < 0.9:
            b["request.path"] = "/api/v%d/%s" % (rng.integers(0, 4), ["reviews", "Ratings", "details"][i % 3])
        if rng.random() < 0.8:
            b["request.headers"] = {"x-forwarded-for": ["10.1.2.%d" % rng.integers(0, 256), "fe80::%x" % rng.integers(0, 65536),
                                                        "bogus"][int(rng.integers(0, 3))]}
        bags.append(b)
    manifest = {"source.labels": "STRING_MAP", "request.path": "STRING", "request.headers": "STRING_MAP"}
    return manifest, BagBatch.from_bags(bags, names=list(manifest))


@pytest.mark.parametrize("case", ["listcheck.yaml", "regex-path", "ci-path", "ip-header"])
def test_listentry_fused(eng, case):
    """mxp_listentry_check: the listentry instance's `value` expression evaluated and checked against
    the list in one device pass (template.gen.go:2153-2202 -> list.go:68-101), against the oracle
    evaluator's Eval feeding the list restatement; eval failures carry the reference's error text."""
    import oracle
    import istio_amd.engine as mxp
    manifest, batch = _listentry_bags(3000, seed=len(case) * 7 + 1)
    if case == "listcheck.yaml":  # mixer/testdata/config/listcheck.yaml: staticversion / appversion
        expr, ltype, entries, overrides, black = 'source.labels["version"]', L.STRINGS, [], ["v1", "v2"], False
        ref = L.StringList([], overrides)
    elif case == "regex-path":
        expr, ltype, entries, overrides, black = 'request.path | "none"', L.REGEX, ["^/api/v[12]/", "details$"], [], True
        ref = L.RegexList(entries)
    elif case == "ci-path":
        expr, ltype, entries, overrides, black = 'request.path', L.CASE_INSENSITIVE_STRINGS, ["/API/V1/RATINGS", "/api/v2/reviews"], [], False
        ref = L.StringList(entries, case_insensitive=True)
    else:
        expr, ltype, entries, overrides, black = 'request.headers["x-forwarded-for"]', L.IP_ADDRESSES, ["10.1.2.0/25", "fe80::/112"], [], True
        ref = L.IPList(entries)
    inst = mxp.Engine(0)
    inst.set_vocabulary(manifest)
    assert (inst.compile(["true", expr]) == 0).all()  # the value expression is rule 1
    lst = eng.list_create(ltype, entries, overrides)
    got, texts = lst.check_entries(inst, batch, 1, black, texts=True)
    ev = oracle.OracleEvaluator(manifest)
    vals, syms, errq = [], [], []
    for q in range(batch.n):
        st, v = ev.eval(expr, batch, q)
        if st != "ok":
            errq.append(q)
            syms.append("")
        else:
            syms.append(v)
    want = L.codes(ref.found(syms), black)
    want[errq] = -1
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(q), syms[q], int(got[q]), int(want[q])) for q in bad[:5]]
    assert (len(errq) > 0) == (case != "regex-path") and (got >= 0).sum() > batch.n // 2  # `|` never fails
    for q in errq[:50]:
        assert inst.pair_error(q, 1) == ev.eval(expr, batch, q)[1]
    # the symbol the status messages print ("%s is not whitelisted", list.go:84-94)
    assert all(texts[q].encode("utf-8", "surrogateescape") == syms[q].encode("utf-8", "surrogateescape")
               for q in range(batch.n) if got[q] >= 0)
    assert all(texts[q] is None for q in errq)


@pytest.mark.parametrize("blacklist", [False, True])
def test_case_insensitive_unicode_parity(eng, blacklist):
    """Case-insensitive lists with non-ASCII and invalid-UTF-8 entries and symbols: Go 1.9's
    strings.ToUpper on both sides (stringList.go:59,66,79; goupper.h on the host and in the kernel)
    against the oracle's restatement -- codes per symbol and numEntries (entries that upper-case to
    one key count once)."""
    entries, syms = W.ci_unicode_list(n_entries=3000, n_lookups=40000, seed=41)
    lst = eng.list_create(L.CASE_INSENSITIVE_STRINGS, entries[:2500] + [""], entries[2500:])
    ref = L.StringList(entries[:2500] + [""], entries[2500:], case_insensitive=True)
    assert lst.num_entries() == ref.num_entries() < len(set(entries))
    want = L.codes(ref.found(syms), blacklist)
    got = lst.check(syms, blacklist)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(syms[i].encode("utf-8", "surrogateescape"), int(got[i]), int(want[i])) for i in bad[:5]]
    hit = 7 if blacklist else 0
    assert (want == hit).sum() > 5000 and (want != hit).sum() > 5000
    # symbols that only match through a non-ASCII mapping ("é" -> "É", "ı" -> "I", "ſ" -> "S")
    assert list(lst.check(["été", "pın", "ſa"], blacklist)) == list(L.codes(ref.found(["été", "pın", "ſa"]), blacklist))


def test_listentry_fused_unicode(eng):
    """The fused listentry path (symbols read from the engine's string pools) on non-ASCII and
    invalid-UTF-8 values, case-insensitive list."""
    import oracle
    import istio_amd.engine as mxp
    from istio_amd.bags import BagBatch
    entries, syms = W.ci_unicode_list(n_entries=1500, n_lookups=6000, seed=43)
    rng = np.random.default_rng(44)
    bags = [{"request.path": s} if rng.random() < 0.95 else {} for s in syms]
    manifest = {"request.path": "STRING"}
    batch = BagBatch.from_bags(bags, names=list(manifest))
    inst = mxp.Engine(0)
    inst.set_vocabulary(manifest)
    assert (inst.compile(["true", "request.path"]) == 0).all()
    lst = eng.list_create(L.CASE_INSENSITIVE_STRINGS, entries, [])
    got, texts = lst.check_entries(inst, batch, 1, False, texts=True)
    ev = oracle.OracleEvaluator(manifest)
    ref = L.StringList(entries, case_insensitive=True)
    want = np.empty(batch.n, dtype=np.int32)
    for q in range(batch.n):
        st, v = ev.eval("request.path", batch, q)
        want[q] = -1 if st != "ok" else L.codes(ref.found([v]), False)[0]
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(q), int(got[q]), int(want[q])) for q in bad[:5]]
    assert (want == 0).sum() > 1000 and (want == -1).sum() > 100
    enc = lambda x: x.encode("utf-8", "surrogateescape")  # noqa: E731 (escaped bytes may re-decode as runes)
    assert all(enc(texts[q]) == enc(bags[q]["request.path"]) for q in range(batch.n) if got[q] >= 0)


RXP_PATTERNS = ["^kk", "^abc$", "\\Aabc.*z", "^abc(?i)def", "^abc\\b", "^abc\\n?$", "^abc.", "(?m)^abd",
                "^k|^j", "^x[0-9]", "^xy[0-9]", "^é[a-z]+$", "^ü", "^qqq[^\\x00-\\x{10FFFF}]",
                "^" + "l" * 40 + "[0-9]", "^" + "m" * 27 + "é[0-9]", "^caf(é|e)s?$", "^tail[a-z]{0,20}$",
                "^z(y|x)w", "^zywv+$"] + ["^shared[0-9]{%d}$" % k for k in range(70)]
RXP_SYMBOLS = ["", "a", "ab", "abx", "k", "kk", "kkx", "j", "jj", "ak", "abc", "abcx", "abcz", "abczz", "abcDEF", "abcdef", "abc def", "abc\n", "abc\n\n",
               "abcé", "abd", "x\nabd", "b", "bb", "x1", "xy1", "xyz", "é", "éabc", "éé", "éab1", "ü", "ab\udcff",
               "qqq", "qqqa", "l" * 40 + "1", "l" * 40, "l" * 39 + "1", "m" * 27 + "é1", "m" * 27 + "e1", "cafés",
               "cafe", "cafés!", "tail" + "a" * 20, "tail" + "a" * 21, "tail" + "a" * 20 + "1", "zyw", "zxw", "zywvvv",
               "zywvx"] + ["shared" + "7" * k for k in range(72)] + ["shared" + "7" * k + "x" for k in range(5)]


def test_regex_list_prefix_dispatch(eng, monkeypatch):
    """Literal-prefix dispatch (lists.cpp rxp_block, mxp_list_rxp_kernel) against the union parts
    (MXP_LIST_RXP=0) and the oracle: prefixes of 1 .. 28+ bytes (longer ones cut at a rune boundary),
    non-ASCII prefixes and tails, tails that only the union can take (`^abc.`), patterns with no
    required prefix ((?m)^, alternation), one that can never match, 70 patterns sharing a prefix (63
    tails a slot), symbols shorter than the prefixes, longer than 32 bytes, with invalid UTF-8; plus
    the C3 list with these mixed in, whitelist and blacklist."""
    rng = np.random.default_rng(91)
    pats, syms = W.c3_regex_list(n_patterns=3000, n_lookups=70_001, seed=92)
    pats = pats[:1500] + RXP_PATTERNS + pats[1500:]
    syms = RXP_SYMBOLS + syms
    out = {}
    for rxp in ("1", "0"):
        monkeypatch.setenv("MXP_LIST_RXP", rxp)
        lst = eng.list_create(L.REGEX, pats, ["^ovr[0-9]$", "(?i)^CASE"])
        out[rxp] = (lst.check(syms + ["ovr1", "case", "CASEx"]), lst.check(syms, True), lst.regex_parts())
    assert out["1"][2][0] < out["0"][2][0] or out["0"][2][0] == 1  # (fewer union parts with the dispatch)
    assert np.array_equal(out["1"][0], out["0"][0]) and np.array_equal(out["1"][1], out["0"][1])
    sample = list(range(len(RXP_SYMBOLS))) + list(len(RXP_SYMBOLS) + rng.choice(len(syms) - len(RXP_SYMBOLS), 600,
                                                                                 replace=False))
    ref = L.RegexList(pats, ["^ovr[0-9]$", "(?i)^CASE"])
    want = L.codes(ref.found([syms[i] for i in sample], threads=16), False)
    bad = [(syms[sample[j]], int(out["1"][0][sample[j]]), int(want[j])) for j in range(len(sample))
           if out["1"][0][sample[j]] != want[j]]
    assert not bad, bad[:8]
    assert (want == 0).sum() > 100 and (want == 5).sum() > 100
