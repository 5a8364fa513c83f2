"""ORACLE (test infrastructure only) -- restatement of Go's regexp.MatchString (RE2 syntax).

Go 1.9's regexp / regexp/syntax (the reference's pinned toolchain; not vendored under
/root/reference) is what the reference calls for `matches` (mixer/pkg/il/runtime/externs.go:118-120,
regexp.MatchString(pattern, str): compile, then an unanchored search) and for regex lists
(mixer/adapter/list/regexList.go:26-65, regexp.Compile + MatchString).  Restated here:

  parse     regexp/syntax parse.go with the flags regexp.Compile uses (syntax.Perl = ClassNL |
            OneLine | PerlX | UnicodeGroups): literals, `.`, classes (ranges, negation, Perl \\d \\s
            \\w and POSIX [:name:] classes), groups ((?flags) (?flags:re) (?:re) (?P<name>re)),
            alternation, * + ? {n} {n,} {n,m} (and their lazy forms), ^ $ \\A \\z \\b \\B, escapes
            (\\a \\f \\t \\n \\r \\v, octal, \\x, \\Q..\\E, punctuation), the i m s U flags, and the
            error codes / texts of syntax.Error ("error parsing regexp: <code>: `<expr>`");
  match     a Pike-VM simulation over the subject decoded the way regexp's inputString does
            (utf8.DecodeRuneInString; an invalid byte is U+FFFD of width 1) with Go's empty-width
            assertions (begin/end line and text, ASCII word boundary).

Unicode classes (\\p{..} / \\P{..}: unicode.Categories, unicode.Scripts, "Any") and simple case
folding read the tables tools/gen_unicode_tables.py generates (oracle/unicode_tables.json, Unicode
13 here where Go 1.9 has Unicode 9).  PARITY UNPINNED beyond the reference's own rows (tests.go:
2064-2121, list_test.go:397-431).
"""
from __future__ import annotations

import json
import os

MAX_REPEAT = 1000
MAX_RUNE = 0x10FFFF


class RegexError(Exception):
    """syntax.Error: text = 'error parsing regexp: <code>: `<expr>`'."""

    def __init__(self, code, expr):
        super().__init__("error parsing regexp: %s: `%s`" % (code, expr))
        self.code, self.expr = code, expr


class Unsupported(Exception):
    pass


E_CLASS = "invalid character class"
E_RANGE = "invalid character class range"
E_ESCAPE = "invalid escape sequence"
E_NAMED = "invalid named capture"
E_PERL = "invalid or unsupported Perl syntax"
E_REPEAT_OP = "invalid nested repetition operator"
E_REPEAT_SIZE = "invalid repeat count"
E_UTF8 = "invalid UTF-8"
E_BRACKET = "missing closing ]"
E_PAREN = "missing closing )"
E_REPEAT_ARG = "missing argument to repetition operator"
E_BACKSLASH = "trailing backslash at end of expression"
E_UNEXPECTED_PAREN = "unexpected )"

# empty-width assertion bits (syntax.EmptyOp)
BEGIN_LINE, END_LINE, BEGIN_TEXT, END_TEXT, WORD_B, NO_WORD_B = 1, 2, 4, 8, 16, 32

PERL_CLASSES = {
    "d": [(0x30, 0x39)],
    "s": [(0x09, 0x0A), (0x0C, 0x0D), (0x20, 0x20)],
    "w": [(0x30, 0x39), (0x41, 0x5A), (0x5F, 0x5F), (0x61, 0x7A)],
}
POSIX_CLASSES = {
    "alnum": [(0x30, 0x39), (0x41, 0x5A), (0x61, 0x7A)],
    "alpha": [(0x41, 0x5A), (0x61, 0x7A)],
    "ascii": [(0x00, 0x7F)],
    "blank": [(0x09, 0x09), (0x20, 0x20)],
    "cntrl": [(0x00, 0x1F), (0x7F, 0x7F)],
    "digit": [(0x30, 0x39)],
    "graph": [(0x21, 0x7E)],
    "lower": [(0x61, 0x7A)],
    "print": [(0x20, 0x7E)],
    "punct": [(0x21, 0x2F), (0x3A, 0x40), (0x5B, 0x60), (0x7B, 0x7E)],
    "space": [(0x09, 0x0D), (0x20, 0x20)],
    "upper": [(0x41, 0x5A)],
    "word": [(0x30, 0x39), (0x41, 0x5A), (0x5F, 0x5F), (0x61, 0x7A)],
    "xdigit": [(0x30, 0x39), (0x41, 0x46), (0x61, 0x66)],
}


# ------------------------------------------------------------------------------- rune helpers
def decode_rune(b: bytes, i: int):
    """utf8.DecodeRune: (rune, width); invalid -> (0xFFFD, 1)."""
    c = b[i]
    if c < 0x80:
        return c, 1
    n = len(b) - i
    if 0xC2 <= c <= 0xDF and n >= 2 and 0x80 <= b[i + 1] <= 0xBF:
        return ((c & 0x1F) << 6) | (b[i + 1] & 0x3F), 2
    if 0xE0 <= c <= 0xEF and n >= 3:
        lo, hi = 0x80, 0xBF
        if c == 0xE0:
            lo = 0xA0
        elif c == 0xED:
            hi = 0x9F
        if lo <= b[i + 1] <= hi and 0x80 <= b[i + 2] <= 0xBF:
            return ((c & 0x0F) << 12) | ((b[i + 1] & 0x3F) << 6) | (b[i + 2] & 0x3F), 3
    if 0xF0 <= c <= 0xF4 and n >= 4:
        lo, hi = 0x80, 0xBF
        if c == 0xF0:
            lo = 0x90
        elif c == 0xF4:
            hi = 0x8F
        if lo <= b[i + 1] <= hi and 0x80 <= b[i + 2] <= 0xBF and 0x80 <= b[i + 3] <= 0xBF:
            return (((c & 0x07) << 18) | ((b[i + 1] & 0x3F) << 12) | ((b[i + 2] & 0x3F) << 6)
                    | (b[i + 3] & 0x3F)), 4
    return 0xFFFD, 1


def full_rune_ok(b: bytes, i: int) -> bool:
    """The pattern text must be valid UTF-8 (checkUTF8)."""
    r, w = decode_rune(b, i)
    return not (r == 0xFFFD and w == 1 and b[i:i + 3] != b"\xef\xbf\xbd")


def valid_utf8(b: bytes) -> bool:
    """checkUTF8 (parse.go)."""
    i = 0
    while i < len(b):
        if not full_rune_ok(b, i):
            return False
        i += decode_rune(b, i)[1]
    return True


def is_word(r: int) -> bool:
    return r >= 0 and (0x30 <= r <= 0x39 or 0x41 <= r <= 0x5A or 0x61 <= r <= 0x7A or r == 0x5F)


def norm(ranges):
    rs = sorted((lo, hi) for lo, hi in ranges if lo <= hi)
    out = []
    for lo, hi in rs:
        if out and lo <= out[-1][1] + 1:
            out[-1] = (out[-1][0], max(out[-1][1], hi))
        else:
            out.append((lo, hi))
    return out


def negate(ranges):
    out, nxt = [], 0
    for lo, hi in norm(ranges):
        if lo > nxt:
            out.append((nxt, lo - 1))
        nxt = hi + 1
    if nxt <= MAX_RUNE:
        out.append((nxt, MAX_RUNE))
    return out


_UNI = None


def _uni():
    """(classes: name -> ranges, fold: rune -> next rune of its orbit) from unicode_tables.json."""
    global _UNI
    if _UNI is None:
        d = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "unicode_tables.json")))
        _UNI = ({k: [tuple(r) for r in v] for k, v in d["classes"].items()}, {a: b for a, b in d["fold"]})
    return _UNI


def fold_orbit(r: int):
    """r and the rest of its unicode.SimpleFold orbit."""
    fold = _uni()[1]
    out, x = [r], fold.get(r, r)
    while x != r:
        out.append(x)
        x = fold[x]
    return out


def fold_ranges(ranges):
    """appendFoldedRange over every range: the class closed under simple case folding."""
    fold = _uni()[1]
    rs = norm(ranges)
    out = list(rs)
    import bisect
    starts = [lo for lo, _ in rs]
    for r in fold:
        k = bisect.bisect_right(starts, r) - 1
        if k >= 0 and r <= rs[k][1]:
            out.extend((o, o) for o in fold_orbit(r))
    return norm(out)


def unicode_class(name):
    """unicodeTable (parse.go): "Any", unicode.Categories, unicode.Scripts; None when unknown."""
    if name == "Any":
        return [(0, MAX_RUNE)]
    return _uni()[0].get(name)


# ------------------------------------------------------------------------------- AST
# nodes: ("lit", r, fold) ("class", ranges) ("any",) ("anynl",) ("empty", op) ("cat", [..])
#        ("alt", [..]) ("star"|"plus"|"quest", n) ("rep", n, lo, hi) ("group", n) ("nop",)


class _Parser:
    def __init__(self, src: bytes):
        self.src = src
        self.whole = src.decode("utf-8", "surrogateescape")
        self.i = 0
        self.flags = {"i": False, "m": False, "s": False, "U": False}

    def err(self, code, expr):
        raise RegexError(code, expr)

    def text(self, a, b=None):
        return self.src[a:b].decode("utf-8", "surrogateescape")

    def parse(self):
        return self.parse_alt(top=True)

    def next_rune(self):
        """nextRune: decode at self.i; invalid UTF-8 -> ErrInvalidUTF8 with the rest of the text."""
        if not full_rune_ok(self.src, self.i):
            self.err(E_UTF8, self.text(self.i))
        r, w = decode_rune(self.src, self.i)
        self.i += w
        return r

    # alternation / concatenation with a stack of open groups, parse.go style errors
    def parse_alt(self, top):
        alts = [[]]
        saved = dict(self.flags)
        while self.i < len(self.src):
            c = self.src[self.i]
            if c == ord("|"):
                self.i += 1
                alts.append([])
                continue
            if c == ord(")"):
                if top:
                    self.err(E_UNEXPECTED_PAREN, self.whole)
                break
            self.parse_piece(alts[-1])
        if not top:
            if self.i >= len(self.src):
                self.err(E_PAREN, self.whole)
            self.i += 1  # ')'
            self.flags = saved
        nodes = [("cat", a) for a in alts]
        return nodes[0] if len(nodes) == 1 else ("alt", nodes)

    def parse_piece(self, seq):
        start = self.i
        c = self.src[self.i]
        if c in b"*+?":
            self.i += 1
            self.repeat(seq, chr(c), start)
            return
        if c == ord("{"):
            rep = self.try_repeat()
            if rep is not None:
                lo, hi = rep
                self.repeat(seq, "{", start, lo, hi)
                return
            self.i += 1
            seq.append(self.lit(ord("{")))
            return
        if c == ord("("):
            self.parse_group(seq)
            return
        if c == ord("["):
            seq.append(("class", self.parse_class()))
            return
        if c == ord("."):
            self.i += 1
            seq.append(("any",) if self.flags["s"] else ("anynl",))
            return
        if c == ord("^"):
            self.i += 1
            seq.append(("empty", BEGIN_LINE if self.flags["m"] else BEGIN_TEXT))
            return
        if c == ord("$"):
            self.i += 1
            seq.append(("empty", END_LINE if self.flags["m"] else END_TEXT))
            return
        if c == ord("\\"):
            self.parse_escape_atom(seq)
            return
        seq.append(self.lit(self.next_rune()))

    def lit(self, r):
        if self.flags["i"]:
            orbit = fold_orbit(r)
            if len(orbit) > 1:
                return ("class", norm((o, o) for o in orbit))
        return ("lit", r)

    def repeat(self, seq, op, start, lo=None, hi=None):
        # missing argument: nothing to repeat (start of group / alternative)
        if not seq or seq[-1][0] == "empty_marker":
            self.err(E_REPEAT_ARG, self.text(start, self.i))
        if self.i < len(self.src) and self.src[self.i] == ord("?"):
            self.i += 1  # lazy form (PerlX); irrelevant for a boolean match
        # nested repetition: the next token is another repetition operator
        if self.i < len(self.src) and self.src[self.i] in b"*+?":
            self.err(E_REPEAT_OP, self.text(start, self.i + 1))
        if self.i < len(self.src) and self.src[self.i] == ord("{"):
            save = self.i
            if self.try_repeat() is not None:
                self.err(E_REPEAT_OP, self.text(start, self.i))
            self.i = save
        prev = seq.pop()
        if op == "*":
            seq.append(("star", prev))
        elif op == "+":
            seq.append(("plus", prev))
        elif op == "?":
            seq.append(("quest", prev))
        else:
            seq.append(("rep", prev, lo, hi))

    def try_repeat(self):
        """{n} {n,} {n,m} at self.i -> (lo, hi | -1) and advance, or None (literal '{')."""
        s, j = self.src, self.i + 1
        def num(j):
            k = j
            while k < len(s) and 0x30 <= s[k] <= 0x39:
                k += 1
            if k == j:
                return None, j
            if k - j > 1 and s[j] == 0x30:
                return None, j  # leading zeros not allowed
            v = int(s[j:k])
            return (v if v <= MAX_REPEAT else MAX_REPEAT + 1), k
        lo, j = num(j)
        if lo is None:
            return None
        if j < len(s) and s[j] == ord(","):
            j += 1
            if j < len(s) and s[j] == ord("}"):
                hi = -1
            else:
                hi, j = num(j)
                if hi is None:
                    return None
        else:
            hi = lo
        if j >= len(s) or s[j] != ord("}"):
            return None
        j += 1
        start = self.i
        self.i = j
        if lo > MAX_REPEAT or hi > MAX_REPEAT or (hi >= 0 and lo > hi):
            self.err(E_REPEAT_SIZE, self.text(start, j))
        return lo, hi

    def parse_group(self, seq):
        start = self.i
        s = self.src
        if self.i + 1 < len(s) and s[self.i + 1] == ord("?"):
            # (?P<name>re)
            if s[self.i + 2:self.i + 4] == b"P<":
                end = s.find(b">", self.i + 4)
                if end < 0:
                    self.err(E_NAMED, self.text(start))
                name = s[self.i + 4:end]
                if not name or not all(is_word(c) for c in name):
                    self.err(E_NAMED, self.text(start, end + 1))
                self.i = end + 1
                seq.append(("group", self.parse_alt(top=False)))
                return
            # flags
            j = self.i + 2
            sign, neg, seen = True, False, False
            newf = dict(self.flags)
            while True:
                if j >= len(s):
                    self.err(E_PERL, self.text(start))
                c = chr(s[j])
                j += 1
                if c in "imsU":
                    newf[c] = sign
                    seen = True
                elif c == "-":
                    if neg:
                        self.err(E_PERL, self.text(start, j))
                    neg, sign, seen = True, False, False
                elif c in ":)":
                    if neg and not seen:
                        self.err(E_PERL, self.text(start, j))
                    if c == ")":
                        self.flags = newf  # (?flags): rest of the current group
                        self.i = j
                        return
                    outer = self.flags
                    self.flags = newf
                    self.i = j
                    seq.append(("group", self.parse_alt(top=False)))
                    self.flags = outer
                    return
                else:
                    self.err(E_PERL, self.text(start, j))
        self.i += 1
        seq.append(("group", self.parse_alt(top=False)))

    def group(self, rs, negated):
        """appendGroup: under (?i) the group is folded BEFORE it is negated."""
        if self.flags["i"]:
            rs = fold_ranges(rs)
        return negate(rs) if negated else norm(rs)

    def perl_class(self):
        """parsePerlClassEscape (\\d \\s \\w and negations) or parseUnicodeClass (\\p, \\P) at
        self.i -> the group's ranges, or None."""
        s = self.src
        if self.i + 1 < len(s) and s[self.i] == ord("\\") and chr(s[self.i + 1]) in "dswDSW":
            c = chr(s[self.i + 1])
            self.i += 2
            return self.group(PERL_CLASSES[c.lower()], c.isupper())
        if self.i + 1 < len(s) and s[self.i] == ord("\\") and chr(s[self.i + 1]) in "pP":
            return self.unicode_class()
        return None

    def unicode_class(self):
        """parseUnicodeClass: \\pN, \\p{Name}, \\P.., \\p{^Name}; unknown -> invalid character class range."""
        s = self.src
        start = self.i
        neg = s[self.i + 1] == ord("P")
        self.i += 2
        if self.i < len(s) and s[self.i] == ord("{"):
            end = s.find(b"}", self.i)
            if end < 0:
                if not valid_utf8(s[start:]):
                    self.err(E_UTF8, self.text(start))
                self.err(E_RANGE, self.text(start))
            name = s[self.i + 1:end]
            if not valid_utf8(name):
                self.err(E_UTF8, self.text(self.i + 1, end))
            seq_end = end + 1
        else:
            if self.i < len(s):
                if not full_rune_ok(s, self.i):
                    self.err(E_UTF8, self.text(self.i))
                r, w = decode_rune(s, self.i)
                name = s[self.i:self.i + w]
                seq_end = self.i + w
            else:
                name, seq_end = b"", self.i
        self.i = seq_end
        name = name.decode("utf-8", "surrogateescape")
        if name.startswith("^"):
            neg = not neg
            name = name[1:]
        tab = unicode_class(name) if name else None
        if tab is None:
            self.err(E_RANGE, self.text(start, seq_end))
        return self.group(tab, neg)

    def parse_escape(self):
        """parseEscape (parse.go): one escaped rune at self.i ('\\'); errors carry the text consumed."""
        start = self.i
        s = self.src
        self.i += 1
        if self.i >= len(s):
            self.err(E_BACKSLASH, "")
        c = self.next_rune()
        def fail():
            self.err(E_ESCAPE, self.text(start, self.i))
        if c < 0x80 and not chr(c).isalnum():
            return c
        ch = chr(c)
        if ch in "1234567":
            if self.i >= len(s) or not (0x30 <= s[self.i] <= 0x37):
                fail()
        if ch in "01234567":
            r = c - 0x30
            for _ in range(2):
                if self.i < len(s) and 0x30 <= s[self.i] <= 0x37:
                    r = r * 8 + s[self.i] - 0x30
                    self.i += 1
            return r
        if ch == "x":
            if self.i >= len(s):
                fail()
            c2 = self.next_rune()
            if c2 == ord("{"):
                nhex, r = 0, 0
                while True:
                    if self.i >= len(s):
                        fail()
                    d = self.next_rune()
                    if d == ord("}"):
                        break
                    v = int(chr(d), 16) if d < 0x80 and chr(d) in "0123456789abcdefABCDEF" else -1
                    if v < 0:
                        fail()
                    r = r * 16 + v
                    if r > MAX_RUNE:
                        fail()
                    nhex += 1
                if nhex == 0:
                    fail()
                return r
            x = int(chr(c2), 16) if c2 < 0x80 and chr(c2) in "0123456789abcdefABCDEF" else -1
            c3 = self.next_rune() if self.i < len(s) else 0xFFFD
            y = int(chr(c3), 16) if c3 < 0x80 and chr(c3) in "0123456789abcdefABCDEF" else -1
            if x < 0 or y < 0:
                fail()
            return x * 16 + y
        simple = {"a": 7, "f": 12, "n": 10, "r": 13, "t": 9, "v": 11}
        if ch in simple:
            return simple[ch]
        fail()

    def parse_escape_atom(self, seq):
        s = self.src
        if self.i + 1 < len(s):
            c = chr(s[self.i + 1])
            if c in "AzbB":
                self.i += 2
                seq.append(("empty", {"A": BEGIN_TEXT, "z": END_TEXT, "b": WORD_B, "B": NO_WORD_B}[c]))
                return
            if c == "C":
                self.err(E_ESCAPE, "\\C")
            if c == "Q":
                self.i += 2
                end = s.find(b"\\E", self.i)
                stop = len(s) if end < 0 else end
                while self.i < stop:
                    seq.append(self.lit(self.next_rune()))
                self.i = len(s) if end < 0 else end + 2
                return
        rs = self.perl_class()
        if rs is not None:
            seq.append(("class", rs))
            return
        seq.append(self.lit(self.parse_escape()))

    def parse_class(self):
        s = self.src
        start = self.i
        self.i += 1
        neg = False
        if self.i < len(s) and s[self.i] == ord("^"):
            neg = True
            self.i += 1
        ranges = []
        first = True
        while True:
            if self.i >= len(s):
                self.err(E_BRACKET, self.text(start))
            c = s[self.i]
            if c == ord("]") and not first:
                self.i += 1
                break
            # POSIX class
            if c == ord("[") and s[self.i + 1:self.i + 2] == b":":
                end = s.find(b":]", self.i + 2)
                if end >= 0:
                    name = s[self.i + 2:end].decode("ascii", "replace")
                    pneg = name.startswith("^")
                    if pneg:
                        name = name[1:]
                    if name not in POSIX_CLASSES:
                        self.err(E_RANGE, self.text(self.i, end + 2))
                    ranges += self.group(POSIX_CLASSES[name], pneg)
                    self.i = end + 2
                    first = False
                    continue
            rs = self.perl_class()
            if rs is not None:
                ranges += rs
                first = False
                continue
            rstart = self.i
            lo = self.class_char(start)
            # range a-b (a trailing '-' before ']' is literal)
            if self.i + 1 < len(s) and s[self.i] == ord("-") and s[self.i + 1] != ord("]"):
                self.i += 1
                hi = self.class_char(start)
                if hi < lo:
                    self.err(E_RANGE, self.text(rstart, self.i))
                ranges.append((lo, hi))
            else:
                ranges.append((lo, lo))
            first = False
        if self.flags["i"]:
            ranges = fold_ranges(ranges)
        ranges = norm(ranges)
        return negate(ranges) if neg else ranges

    def class_char(self, class_start):
        """parseClassChar: end of text -> missing ']' (the whole class), escape, or a rune."""
        s = self.src
        if self.i >= len(s):
            self.err(E_BRACKET, self.text(class_start))
        if s[self.i] == ord("\\"):
            return self.parse_escape()
        return self.next_rune()


def parse(pattern) -> tuple:
    src = pattern.encode("utf-8", "surrogateescape") if isinstance(pattern, str) else bytes(pattern)
    return _Parser(src).parse()


# ------------------------------------------------------------------------------- NFA (Pike VM)
class Prog:
    """Instructions: ("rune", ranges, next) ("split", a, b) ("empty", op, next) ("match",)."""

    def __init__(self):
        self.ins = []

    def emit(self, x):
        self.ins.append(list(x))
        return len(self.ins) - 1


def _compile(p: Prog, n, nxt):
    """Compile node n so that it continues at pc `nxt`; returns its entry pc."""
    k = n[0]
    if k == "lit":
        return p.emit(("rune", [(n[1], n[1])], nxt))
    if k == "class":
        return p.emit(("rune", n[1], nxt))
    if k == "any":
        return p.emit(("rune", [(0, MAX_RUNE)], nxt))
    if k == "anynl":
        return p.emit(("rune", [(0, 9), (11, MAX_RUNE)], nxt))
    if k == "empty":
        return p.emit(("empty", n[1], nxt))
    if k == "group":
        return _compile(p, n[1], nxt)
    if k == "cat":
        pc = nxt
        for c in reversed(n[1]):
            pc = _compile(p, c, pc)
        return pc
    if k == "alt":
        entries = [_compile(p, c, nxt) for c in n[1]]
        pc = entries[-1]
        for e in reversed(entries[:-1]):
            pc = p.emit(("split", e, pc))
        return pc
    if k == "quest":
        body = _compile(p, n[1], nxt)
        return p.emit(("split", body, nxt))
    if k == "star":
        loop = p.emit(("split", -1, nxt))
        body = _compile(p, n[1], loop)
        p.ins[loop][1] = body
        return loop
    if k == "plus":
        loop = p.emit(("split", -1, nxt))
        body = _compile(p, n[1], loop)
        p.ins[loop][1] = body
        return body
    if k == "rep":
        _, sub, lo, hi = n
        pc = nxt
        if hi < 0:
            pc = _compile(p, ("star", sub), pc)
        else:
            for _ in range(hi - lo):
                body = _compile(p, sub, pc)
                pc = p.emit(("split", body, pc))
        for _ in range(lo):
            pc = _compile(p, sub, pc)
        return pc
    raise AssertionError(k)


def compile(pattern):
    """regexp.Compile: raises RegexError (Go's message) or Unsupported."""
    ast = parse(pattern)
    p = Prog()
    m = p.emit(("match",))
    p.start = _compile(p, ast, m)
    return p


def _flags(prev, nxt):
    f = 0
    if prev < 0:
        f |= BEGIN_TEXT | BEGIN_LINE
    elif prev == 10:
        f |= BEGIN_LINE
    if nxt < 0:
        f |= END_TEXT | END_LINE
    elif nxt == 10:
        f |= END_LINE
    if is_word(prev) != is_word(nxt):
        f |= WORD_B
    else:
        f |= NO_WORD_B
    return f


def match(prog: Prog, subject) -> bool:
    """regexp.(*Regexp).MatchString: unanchored search, any match."""
    b = subject.encode("utf-8", "surrogateescape") if isinstance(subject, str) else bytes(subject)
    runes = []
    i = 0
    while i < len(b):
        r, w = decode_rune(b, i)
        runes.append(r)
        i += w
    ins = prog.ins

    def add(pcs, pc, flags, seen):
        stack = [pc]
        while stack:
            pc = stack.pop()
            if pc in seen:
                continue
            seen.add(pc)
            x = ins[pc]
            if x[0] == "split":
                stack.append(x[2])
                stack.append(x[1])
            elif x[0] == "empty":
                if x[1] & flags == x[1]:
                    stack.append(x[2])
            else:
                pcs.append(pc)

    clist = []
    for pos in range(len(runes) + 1):
        prev = runes[pos - 1] if pos > 0 else -1
        nxt = runes[pos] if pos < len(runes) else -1
        flags = _flags(prev, nxt)
        seen = set()
        cur = []
        for pc in clist:  # threads that consumed the previous rune: re-close under this position's flags
            add(cur, pc, flags, seen)
        add(cur, prog.start, flags, seen)  # unanchored: a new thread at every position
        if any(ins[pc][0] == "match" for pc in cur):
            return True
        if nxt < 0:
            return False
        clist = []
        for pc in cur:
            x = ins[pc]
            if x[0] == "rune" and any(lo <= nxt <= hi for lo, hi in x[1]):
                clist.append(x[2])
    return False


def match_string(pattern, subject):
    """(matched, error text or None) as regexp.MatchString(pattern, subject) returns."""
    try:
        p = compile(pattern)
    except RegexError as e:
        return False, str(e)
    return match(p, subject), None
