"""An independent pin for the regex restatements: Python's own `re` engine (sre, a backtracking
matcher written apart from both the oracle and the product) on the syntax subset where Go's
`regexp.MatchString` (mixer/pkg/il/runtime/externs.go:118-120 `match`) and `re.search` agree on
whether a subject matches.  Every other check of Go regexp behaviour beyond the reference's own rows
compares the builder's restatements with each other (oracle/goregex.py, oracle/goregex.c,
istio_amd/csrc/regex.cpp); this one does not.

The subset and its translation (Go -> Python, both under ASCII classes):
  literals, `.`, `[a-c]`, `[^b]`, `\\d`, `\\w`, `\\s`, `\\b`, `\\B`, `\\.`, `\\x{e9}` -> `\\xe9`, `é`,
  `[[:alpha:]]` -> `[A-Za-z]`, groups, alternation, `* + ? {n} {n,m}` and their lazy forms,
  `^` / `\\A`, `$` / `\\z` -> `\\Z` (Go's `$` without (?m) is end of text only), `(?m:^)`,
  `(?m:$)`, `(?s:.)`, `(?i:...)` over ASCII letters.
Subjects avoid the runes where the two differ: U+212A / U+017F (Go's (?i) folds them with k / s)
and U+000B (in Python's ASCII `\\s`, not in Go's).  Invalid UTF-8 is one U+FFFD rune in Go and one
lone surrogate in Python: either way a single non-word, non-digit code point that `.` matches.
One sre quirk is stepped around: before Python 3.14 `\\B` never matches an empty subject (Go's does,
and so do the oracle's and the product's), so patterns holding `\\B` skip the empty subject."""
import re

import numpy as np
import pytest

import goregex as G

# (Go, Python) atoms that consume a character (quantifiable) ...
CHAR_ATOMS = [("a", "a"), ("b", "b"), ("c", "c"), ("x", "x"), (".", "."), ("[a-c]", "[a-c]"), ("[^b]", "[^b]"),
              ("\\d", "\\d"), ("\\w", "\\w"), ("\\s", "\\s"), ("\\.", "\\."), ("\\x{e9}", "\\xe9"), ("é", "é"),
              ("[[:alpha:]]", "[A-Za-z]"), ("(?s:.)", "(?s:.)"), ("(?i:a)", "(?i:a)"), ("(?i:xb)", "(?i:xb)"),
              ("[0-9_]", "[0-9_]"), ("[^\\n]", "[^\\n]"), ("-", "-")]
# ... and empty-width assertions (never quantified: Python refuses `^*`)
ASSERTS = [("^", "^"), ("$", "\\Z"), ("\\A", "\\A"), ("\\z", "\\Z"), ("\\b", "\\b"), ("\\B", "\\B"),
           ("(?m:^)", "(?m:^)"), ("(?m:$)", "(?m:$)")]
QUANTS = ["*", "+", "?", "{2}", "{1,3}", "{0,2}", "*?", "+?", "??"]


def _gen(rng, depth=0):
    go, py = [], []
    for _ in range(int(rng.integers(1, 4))):
        r = rng.random()
        if r < 0.15 and depth < 2:
            g, p = _gen(rng, depth + 1)
            g, p = "(" + g + ")", "(" + p + ")"
        elif r < 0.25 and depth < 2:
            g1, p1 = _gen(rng, depth + 1)
            g2, p2 = _gen(rng, depth + 1)
            g, p = "(?:" + g1 + "|" + g2 + ")", "(?:" + p1 + "|" + p2 + ")"
        elif r < 0.4:
            g, p = ASSERTS[int(rng.integers(len(ASSERTS)))]
            go.append(g)
            py.append(p)
            continue
        else:
            g, p = CHAR_ATOMS[int(rng.integers(len(CHAR_ATOMS)))]
        if rng.random() < 0.35:
            q = QUANTS[int(rng.integers(len(QUANTS)))]
            g, p = "(?:" + g + ")" + q, "(?:" + p + ")" + q
        go.append(g)
        py.append(p)
    return "".join(go), "".join(py)


def _subjects(rng, n):
    alpha = ["a", "b", "c", "x", "X", "A", "B", "1", "_", " ", "\n", "\t", ".", "-", "é", "É", "z", "\udcff"]
    return ["".join(alpha[int(i)] for i in rng.integers(0, len(alpha), size=int(rng.integers(0, 10))))
            for _ in range(n)]


def _cases(seed, n_pats, n_subj):
    rng = np.random.default_rng(seed)
    pats = [_gen(rng) for _ in range(n_pats)]
    return pats, _subjects(rng, n_subj) + ["", "\n", "a\n", "\na"]


@pytest.mark.parametrize("seed", [11, 12])
def test_oracle_matches_python_re(seed):
    pats, subs = _cases(seed, 250, 40)
    for go, py in pats:
        prog = G.compile(go)  # every generated pattern is valid Go syntax
        cre = re.compile(py, re.ASCII)
        for s in subs:
            if not s and "\\B" in py:
                continue
            assert G.match(prog, s) == (cre.search(s) is not None), (go, py, s)


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_product_matches_python_re(libmxp, seed):
    from istio_amd.engine import regex_match_host
    pats, subs = _cases(seed, 300, 40)
    n_true = 0
    for go, py in pats:
        cre = re.compile(py, re.ASCII)
        for s in subs:
            if not s and "\\B" in py:
                continue
            want = cre.search(s) is not None
            n_true += want
            assert regex_match_host(go, s) == (1 if want else 0, ""), (go, py, s)
    assert 0.1 < n_true / (len(pats) * len(subs)) < 0.9  # (both answers well represented)


@pytest.mark.gpu
@pytest.mark.parametrize("flags", ["0", "262144"])  # 262144: value classes forced
def test_gpu_rules_match_python_re(libmxp, monkeypatch, flags):
    """The same patterns as rule constants (`"<p>".matches(request.path)`, the DFA kernels) and as
    run-time patterns (`x.matches(request.path)`, one pattern per request) on the GPU."""
    import istio_amd.engine as mxp
    from istio_amd.bags import BagBatch
    from test_gpu_parity import gpu_codes
    monkeypatch.setenv("MXP_DEBUG_FLAGS", flags)
    pats, subs = _cases(21, 200, 60)
    pats = [(g, p) for g, p in pats if "\\B" not in p]  # (the sre empty-subject quirk)
    n = 3000
    rng = np.random.default_rng(22)
    pick = rng.integers(0, len(subs), size=n)
    rt = rng.integers(0, len(pats), size=n)
    manifest = {"request.path": "STRING", "x": "STRING"}
    bags = [{"request.path": subs[int(pick[q])], "x": pats[int(rt[q])][0]} for q in range(n)]
    batch = BagBatch.from_bags(bags, names=list(manifest))
    rules = ['"%s".matches(request.path)' % g.replace("\\", "\\\\") for g, _ in pats] + ["x.matches(request.path)"]
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    st = eng.compile(rules)
    assert (st == 0).all(), [eng.rule_error(i) for i in range(len(rules)) if st[i]]
    got = gpu_codes(eng, batch)
    cres = [re.compile(p, re.ASCII) for _, p in pats]
    want = np.array([[cre.search(subs[int(pick[q])]) is not None for cre in cres] +
                     [cres[int(rt[q])].search(subs[int(pick[q])]) is not None] for q in range(n)], dtype=got.dtype)
    bad = np.argwhere(got != want)
    assert bad.size == 0, [(int(q), rules[r], subs[int(pick[q])], int(got[q, r]), int(want[q, r])) for q, r in bad[:5]]
    assert 0.1 < want.mean() < 0.9
