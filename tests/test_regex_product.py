"""The engine's regex compiler (istio_amd/csrc/regex.cpp: Go regexp parse -> NFA -> DFA), stepped on
the host through mxp_regex_match_host, against the oracle restatement (oracle/goregex.py): every
known-answer, error and Unicode case of tests/test_regex_oracle.py plus seeded random patterns
over random subjects.  The GPU kernels step these same DFA tables (test_gpu_regex.py)."""
import numpy as np
import pytest

import goregex as G
from test_regex_oracle import ERRORS, GOLDEN, KAT, UNICODE_ERRORS, UNICODE_KAT


@pytest.fixture(scope="module")
def rx(libmxp):
    from istio_amd.engine import regex_match_host
    return regex_match_host


def test_known_answers_and_golden(rx):
    for pat, subj, want in GOLDEN + KAT:
        assert rx(pat, subj) == (1 if want else 0, ""), (pat, subj)


def test_error_texts(rx):
    for pat, msg in ERRORS:
        assert rx(pat, "") == (-1, "error parsing regexp: " + msg), pat


def test_unicode_classes_and_folding(rx):
    for pat, subj, want in UNICODE_KAT:
        assert rx(pat, subj) == (1 if want else 0, ""), (pat, subj)
    for pat, msg in UNICODE_ERRORS:
        assert rx(pat, "") == (-1, "error parsing regexp: " + msg), pat


ATOMS = ["a", "b", "ab", ".", "[a-c]", "[^b]", "\\d", "\\w", "\\s", "\\b", "\\B", "^", "$", "(?i:a)", "(a|b)",
         "(?:ab|ba)", "a*", "b+", "c?", "x{2}", "a{1,2}", "[[:alpha:]]", "\\.", "é", "\\x{e9}", "(?s:.)", "(?m:^)",
         "(?m:$)", "\\Aa", "a\\z", "[a-]", "k", "(?i)k", "\\pL", "\\p{Greek}+", "\\P{L}", "(?i)σ", "(?i)[à-ÿ]",
         "[\\p{Nd}_]", "(?i)\\W", "\\p{Lu}\\p{Ll}"]


def random_patterns(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        k = int(rng.integers(1, 5))
        parts = [ATOMS[int(rng.integers(len(ATOMS)))] for _ in range(k)]
        p = "".join(parts)
        r = rng.random()
        if r < 0.2:
            p = "(" + p + ")*"
        elif r < 0.3:
            p = p + "|" + ATOMS[int(rng.integers(len(ATOMS)))]
        elif r < 0.35:
            p = p + "**"  # syntax error
        out.append(p)
    return out


def random_subjects(n, seed):
    rng = np.random.default_rng(seed)
    alpha = ["a", "b", "c", "x", "1", " ", "\n", ".", "é", "K", "K", "_", "\udcff", "-"]
    return ["".join(alpha[int(i)] for i in rng.integers(0, len(alpha), size=int(rng.integers(0, 9))))
            for _ in range(n)]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_patterns_match_oracle(rx, seed):
    pats = random_patterns(120, seed)
    subs = random_subjects(60, seed + 100)
    for p in pats:
        try:
            prog = G.compile(p)
        except G.RegexError as e:
            assert rx(p, "") == (-1, str(e)), p
            continue
        for s in subs:
            want = G.match(prog, s)
            got = rx(p, s)
            assert got == (1 if want else 0, ""), (p, s, got, want)


# Patterns whose DFA is over the rules' 65,536-state budget: the bit-parallel NFA (regex.cpp
# build_nfa; the device walks the same image, dfa_dev.h mxp_nfa_run), against the C oracle.
NFA_PATTERNS = ["(a|b)*a(a|b){16}", "^(a|b)*b(a|b){17}$", "(?m)^x.{16}y$", "\\b[ab]*a[ab]{16}\\b", "(?i)é.{16}z",
                "(a|b)*a(a|b){15}(c|$)", "[^x]*x.{20}\\z", "é[\\pL ]{16}\\PL"]


def _nfa_subjects(rng, n):
    alpha = ["a", "b", "x", "y", "z", "é", "É", "\n", " ", "c", "1"]
    w = np.array([8, 8, 2, 1, 1, 1, 1, 1, 1, 1, 1], dtype=float)
    out = []
    for _ in range(n):
        L = int(rng.integers(0, 48))
        out.append("".join(rng.choice(alpha, size=L, p=w / w.sum())))
    return out


def test_over_budget_patterns_walk_the_nfa(rx):
    import oracle
    rng = np.random.default_rng(9)
    subs = _nfa_subjects(rng, 400) + ["a" + "b" * 16, "b" * 18 + "a" + "a" * 16, "x" + "0" * 16 + "y", ""]
    for p in NFA_PATTERNS:
        n_true = 0
        for s in subs:
            want = oracle.regex_match(p, s)
            assert want[0] in (0, 1), (p, want)
            got = rx(p, s)
            assert got == want, (p, s, got, want)
            n_true += got[0]
        assert 0 < n_true < len(subs), p


def wide_subjects(rng, n, tail):
    """Subjects for the wide-NFA patterns `(a|b)*a(a|b){16}` + tail: half built to match."""
    out = []
    for i in range(n):
        s = "".join(rng.choice(["a", "b"], size=int(rng.integers(0, 20)))) + "a"
        s += "".join(rng.choice(["a", "b"], size=16)) + tail
        if i % 2:  # a near miss: a wrong byte somewhere in the tail, or the tail cut short
            k = int(rng.integers(0, len(tail) + 1))
            s = s[:len(s) - len(tail) + k] + ("x" if i % 4 == 1 else "")
        out.append(s)
    return out


def test_nfa_wide_programs(rx):
    """Over budget and wider than 255 rune instructions: the wide NFA walks (private-memory thread
    sets up to 1023 rune instructions, global-memory ones up to 16319) against the oracle; only a
    program wider than that is refused (-3, err says why)."""
    import oracle
    rng = np.random.default_rng(19)
    for tail in ("c" * 260, "cd" * 300 + "e" * 200, "c" * 1100):
        p = "(a|b)*a(a|b){16}" + tail
        subs = wide_subjects(rng, 60, tail)
        hits = 0
        for sub in subs:
            want = oracle.regex_match(p, sub)
            assert rx(p, sub) == want, (p[:30], sub[:40])
            hits += want[0]
        assert 0 < hits < len(subs)
    rc, err = rx("(a|b)*a(a|b){16}" + "c" * 16400, "ab")
    assert rc == -3 and "NFA" in err


def test_over_budget_rules_compile(libmxp):
    """Rule compile (host-only engine): over-budget constant patterns are accepted (their rules walk
    the NFA); only an over-budget pattern wider than the NFA is refused, naming why."""
    from istio_amd.engine import Engine
    eng = Engine(-1)
    eng.set_vocabulary({"request.path": "STRING"})
    rules = ['"%s".matches(request.path)' % p.replace("\\", "\\\\") for p in NFA_PATTERNS]
    rules.append('"(a|b)*a(a|b){16}%s".matches(request.path)' % ("c" * 260))   # wide NFA: compiles
    rules.append('"(a|b)*a(a|b){16}%s".matches(request.path)' % ("c" * 1100))  # global thread sets: compiles
    rules.append('"(a|b)*a(a|b){16}%s".matches(request.path)' % ("c" * 16400))  # wider than 16319: refused
    st = eng.compile(rules)
    assert (st[:-1] == 0).all(), [eng.rule_error(i) for i in range(len(rules) - 1) if st[i]]
    assert st[-1] != 0 and "NFA" in eng.rule_error(len(rules) - 1)
