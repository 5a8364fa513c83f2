"""strings.ToUpper for case-insensitive lists (stringList.go:59,66,79): the engine's mxp_go_to_upper
(istio_amd/csrc/goupper.h, the code the list kernel runs per symbol) against the oracle's restatement
(oracle/lists.py go_to_upper) and known answers of Go 1.9's unicode.ToUpper (Unicode 9.0.0 simple
uppercase, UnicodeData.txt field 12).  No reference fixture covers non-ASCII symbols: beyond these
known answers parity is unpinned (the two tables are derived independently from the image's UCD)."""
import json
import os

import numpy as np
import pytest

import lists as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# unicode.ToUpper known answers (Unicode 9.0.0 UnicodeData.txt simple uppercase mappings)
KAT = {
    0x61: 0x41, 0x7A: 0x5A, 0x41: 0x41, 0xE9: 0xC9, 0xDF: 0xDF, 0xFF: 0x178, 0x131: 0x49, 0x17F: 0x53,
    0xB5: 0x39C, 0x1C4: 0x1C4, 0x1C5: 0x1C4, 0x1C6: 0x1C4, 0x345: 0x399, 0x3C2: 0x3A3, 0x1E9E: 0x1E9E,
    0x1E9B: 0x1E60, 0x1F80: 0x1F88, 0x1FB3: 0x1FBC, 0x24D0: 0x24B6, 0xFF41: 0xFF21, 0x10428: 0x10400,
    0x104D8: 0x104B0, 0x1E922: 0x1E900, 0xAB70: 0x13A0, 0x13F8: 0x13F0, 0x250: 0x2C6F, 0x2C65: 0x23A,
    0x587: 0x587, 0x149: 0x149, 0x1F0: 0x1F0, 0x212A: 0x212A, 0x2126: 0x2126, 0x130: 0x130, 0x1D79: 0xA77D,
    0x265: 0xA78D, 0x26A: 0xA7AE, 0x29D: 0xA7B2, 0xAB53: 0xA7B3, 0x1C80: 0x412, 0x1C88: 0xA64A,
    0x101: 0x100, 0x100: 0x100, 0x3B1: 0x391, 0x430: 0x410, 0x561: 0x531, 0x1E01: 0x1E00,
    # capitals Unicode 11-12 added for runes of 9.0: no mapping in Go 1.9's tables
    0x10D0: 0x10D0, 0x10FA: 0x10FA, 0xA794: 0xA794, 0x282: 0x282, 0x1D8E: 0x1D8E,
    # unassigned in 9.0 (Latin 11.0, Medefaidrin 11.0); Old Hungarian is 8.0
    0xA7B9: 0xA7B9, 0x16E60: 0x16E60, 0x10CC0: 0x10C80,
}


def enc(r):
    return chr(r).encode("utf-8", "surrogatepass")


@pytest.fixture(scope="module")
def up(libmxp):
    from istio_amd.engine import go_to_upper
    return go_to_upper


def test_known_answers_oracle():
    for r, u in KAT.items():
        assert L.go_upper_rune(r) == u, hex(r)
        assert L.go_to_upper(enc(r)) == enc(u), hex(r)


def test_known_answers_engine(up):
    for r, u in KAT.items():
        assert up(enc(r)) == enc(u), hex(r)


def test_every_rune_engine_equals_oracle(up):
    """All runes re-encoded after a leading 'a' (which switches strings.Map to re-encoding): one call
    covers the engine's whole table; surrogate code points are invalid UTF-8 (three U+FFFD each)."""
    s = b"a" + b"".join(enc(r) for r in range(0x80, 0x110000))
    got, want = up(s), L.go_to_upper(s)
    assert len(got) == len(want)
    if got != want:
        k = next(i for i in range(len(got)) if got[i] != want[i])
        pytest.fail("first difference at byte %d: %r vs %r" % (k, got[k - 8:k + 8], want[k - 8:k + 8]))
    assert L.go_to_upper(b"".join(enc(r) for r in range(0x80, 0x800))) != b"".join(enc(r) for r in range(0x80, 0x800))


def test_oracle_table_agrees_with_engine_table():
    """The two independently generated tables (tools/gen_upper_table.py range rows vs
    tools/gen_oracle_upper.py per code point) hold the same mapping."""
    import re
    txt = open(os.path.join(ROOT, "istio_amd", "csrc", "upper_table.h")).read()
    rows = [tuple(int(x, 16) for x in m) for m in re.findall(r"\{0x([0-9A-F]+), 0x([0-9A-F]+), 0x([0-9A-F]+)\}", txt)]
    eng = {}
    for lo, hi, d in rows:
        for r in range(lo, hi + 1):
            u = lo + ((r - lo) & ~1) if d == 0x80000000 else (r + d) & 0xFFFFFFFF
            if u != r:
                eng[r] = u
    orc = {a: b for a, b in json.load(open(os.path.join(ROOT, "oracle", "unicode_upper.json")))["pairs"]}
    orc.update({r: r - 32 for r in range(0x61, 0x7B)})
    assert eng == orc


# strings.Map semantics around invalid UTF-8: bytes before the first changing rune stay as they are,
# every rune after it is EncodeRune'd (an invalid byte becomes EF BF BD)
MAP_CASES = [
    (b"", b""), (b"ABC", b"ABC"), (b"abc", b"ABC"), (b"ABC\xff", b"ABC\xff"), (b"\xffabc", b"\xffABC"),
    (b"abc\xff", b"ABC\xef\xbf\xbd"), (b"\xe2\x82", b"\xe2\x82"), (b"a\xe2\x82", b"A\xef\xbf\xbd\xef\xbf\xbd"),
    (b"a\xc0\x80", b"A\xef\xbf\xbd\xef\xbf\xbd"), (b"a\xed\xa0\x80", b"A" + b"\xef\xbf\xbd" * 3),
    (b"a\xf4\x8f\xbf\xbf", b"A\xf4\x8f\xbf\xbf"), (b"a\xf4\x90\x80\x80", b"A" + b"\xef\xbf\xbd" * 4),
    (b"\xef\xbf\xbdb", b"\xef\xbf\xbdB"), ("été".encode(), "ÉTÉ".encode()), ("ÉTÉ".encode(), "ÉTÉ".encode()),
    ("straße".encode(), "STRAßE".encode()), ("ı".encode(), b"I"), ("ɐ".encode(), "Ɐ".encode()),
    (b"x" * 9 + "é".encode() * 5, b"X" * 9 + "É".encode() * 5),
]


@pytest.mark.parametrize("s,want", MAP_CASES)
def test_map_semantics(up, s, want):
    assert L.go_to_upper(s) == want
    assert up(s) == want


def test_random_bytes_engine_equals_oracle(up):
    rng = np.random.default_rng(5)
    alphabet = [b"a", b"Z", b"\xff", b"\xc3", b"\xa9", b"\xe2\x82", "é".encode(), "ı".encode(), "ß".encode(),
                "ᾀ".encode(), "\U0001e922".encode(), b"\xf0\x90", "ǅ".encode(), b"\x80", b"0"]
    for _ in range(4000):
        s = b"".join(alphabet[i] for i in rng.integers(0, len(alphabet), rng.integers(0, 14)))
        assert up(s) == L.go_to_upper(s), s
