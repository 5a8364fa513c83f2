"""The engine's regex compiler (istio_amd/csrc/regex.cpp: Go regexp parse -> NFA -> DFA), stepped on
the host through mxp_regex_match_host, against the oracle restatement (oracle/goregex.py): every
known-answer, error and unsupported case of tests/test_regex_oracle.py plus seeded random patterns
over random subjects.  The GPU kernels step these same DFA tables (test_gpu_regex.py)."""
import numpy as np
import pytest

import goregex as G
from test_regex_oracle import ERRORS, GOLDEN, KAT


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


def test_unsupported(rx):
    for pat in ["\\pL", "\\p{Greek}", "(?i)é", "(?i)[à-ÿ]"]:
        assert rx(pat, "x")[0] == -2, pat
    assert rx("(?i)\\W", "k") == (1, "")


ATOMS = ["a", "b", "ab", ".", "[a-c]", "[^b]", "\\d", "\\w", "\\s", "\\b", "\\B", "^", "$", "(?i:a)", "(a|b)",
         "(?:ab|ba)", "a*", "b+", "c?", "x{2}", "a{1,2}", "[[:alpha:]]", "\\.", "é", "\\x{e9}", "(?s:.)", "(?m:^)",
         "(?m:$)", "\\Aa", "a\\z", "[a-]", "k", "(?i)k"]


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
        except G.Unsupported:
            assert rx(p, "")[0] == -2, p
            continue
        for s in subs:
            want = G.match(prog, s)
            got = rx(p, s)
            assert got == (1 if want else 0, ""), (p, s, got, want)
