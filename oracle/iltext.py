"""ORACLE (test infrastructure only) -- the Mixer IL assembler: text.ReadText / MergeText.

Restates mixer/pkg/il/text/scanner.go:26-338 (the rune-at-a-time token state machine: identifiers,
labels `L0:`, string literals with backslash escapes removed, decimal / hex / float literals, `//`
comments, newlines, parentheses) and mixer/pkg/il/text/read.go:26-377 (`fn name(types) rtype`
headers, opcode bodies up to `end`, label fixups local to the body, registers `rN`), building an
oracle/ilcompile.Program that oracle/il_interp.c runs.  Used to run the reference's IL-level test
table (tests/golden/il_interpreter.json, from interpreter_test.go) through the oracle interpreter.
Not part of the product.
"""
from __future__ import annotations

import unicodedata

import ilcompile as IL

TK_NONE, TK_ERROR, TK_IDENT, TK_STRING, TK_INT, TK_FLOAT, TK_NEWLINE, TK_LABEL, TK_OPEN, TK_CLOSE = range(10)
(SC_SCAN, SC_BEGIN_COMMENT, SC_COMMENT, SC_STRING, SC_STRING_ESC, SC_DEC_HEX_FLOAT, SC_DEC_FLOAT, SC_FLOAT,
 SC_HEX, SC_IDENT_LABEL, SC_END, SC_ERROR) = range(12)


class ReadError(Exception):
    pass


def _is_letter(r):
    return r != 0 and unicodedata.category(chr(r)).startswith("L")


def _is_space(r):
    return r in (0x09, 0x0A, 0x0B, 0x0C, 0x0D, 0x20, 0x85, 0xA0) or (
        r > 0xFF and unicodedata.category(chr(r)) == "Zs")


def _is_digit(r):
    return r != 0 and unicodedata.category(chr(r)) == "Nd"


class _Scanner:
    """scanner.go: next() leaves the token in `token`, its text in raw(); positions in runes of
    `text` (a str), as the reference ranges over the UTF-8 string rune by rune."""

    def __init__(self, text):
        self.text = text
        self.begin = self.current = 0
        self.line, self.col = 1, 1
        self.lbegin = (1, 1)
        self.state = SC_SCAN
        self.token = TK_NONE

    def end(self):
        return self.state in (SC_END, SC_ERROR)

    def next(self):
        if self.end():
            return False
        self.state, self.token = SC_SCAN, TK_NONE
        done = False
        while self.current < len(self.text):
            rn = ord(self.text[self.current])
            done = self._on_rune(rn)
            if done:
                break
            self._advance(rn)
        if not done:
            done = self._on_rune(0)
            if self.state != SC_ERROR:
                self.state = SC_END
        if self.state == SC_ERROR:
            self.token = TK_ERROR
            self.begin = self.current
            self.lbegin = (self.line, self.col)
        return done

    def _advance(self, rn):
        if rn == 0x0A:
            self.line += 1
            self.col = 0
        self.current += 1
        self.col += 1

    def _mark(self):
        self.begin = self.current
        self.lbegin = (self.line, self.col)

    def _on_rune(self, rn):
        st = self.state
        end_ok = lambda: _is_space(rn) or rn == 0x2F or rn == 0  # noqa: E731
        if st == SC_SCAN:
            self._mark()
            c = chr(rn) if rn else "\0"
            if rn == 0:
                pass
            elif c == "\n":
                self.token = TK_NEWLINE
                self._advance(rn)
            elif c == "/":
                self.state = SC_BEGIN_COMMENT
            elif c == '"':
                self.state = SC_STRING
            elif c == "(":
                self.token = TK_OPEN
                self._advance(rn)
            elif c == ")":
                self.token = TK_CLOSE
                self._advance(rn)
            elif c in "0-":
                self.state = SC_DEC_HEX_FLOAT
            elif c in "123456789":
                self.state = SC_DEC_FLOAT
            elif c == ".":
                self.state = SC_FLOAT
            elif _is_letter(rn):
                self.state = SC_IDENT_LABEL
            elif _is_space(rn):
                pass
            else:
                self.state = SC_ERROR
        elif st == SC_BEGIN_COMMENT:
            self.state = SC_COMMENT if rn == 0x2F else SC_ERROR
        elif st == SC_COMMENT:
            if rn == 0x0A:
                self._mark()
                self.token = TK_NEWLINE
                self._advance(rn)
        elif st == SC_STRING:
            if rn == 0x5C:
                self.state = SC_STRING_ESC
            elif rn == 0x22:
                self.token = TK_STRING
                self._advance(rn)
            elif rn in (0x0A, 0):
                self.state = SC_ERROR
        elif st == SC_STRING_ESC:
            self.state = SC_ERROR if rn in (0, 0x0A) else SC_STRING
        elif st == SC_IDENT_LABEL:
            if rn == 0x3A:
                self.token = TK_LABEL
                self._advance(rn)
            elif _is_space(rn) or rn in (0x0A, 0x2F, 0x28, 0x29, 0):
                self.token = TK_IDENT
            elif not _is_digit(rn) and not _is_letter(rn) and rn != 0x5F:
                self.state = SC_ERROR
        elif st == SC_DEC_HEX_FLOAT:
            if 0x30 <= rn <= 0x39:
                self.state = SC_DEC_FLOAT
            elif rn in (0x78, 0x58):
                self.state = SC_HEX
            else:
                self.token = TK_INT
                if not end_ok():
                    self.state = SC_ERROR
        elif st == SC_DEC_FLOAT:
            if 0x30 <= rn <= 0x39:
                pass
            elif rn == 0x2E:
                self.state = SC_FLOAT
            else:
                self.token = TK_INT
                if not end_ok():
                    self.state = SC_ERROR
        elif st == SC_FLOAT:
            if not 0x30 <= rn <= 0x39:
                self.token = TK_FLOAT
                if not end_ok():
                    self.state = SC_ERROR
        elif st == SC_HEX:
            if not (_is_digit(rn) or 0x61 <= rn <= 0x66 or 0x41 <= rn <= 0x46):
                self.token = TK_INT
                if not end_ok():
                    self.state = SC_ERROR
        return self.state == SC_ERROR or self.token != TK_NONE

    def raw(self):
        return self.text[self.begin:self.current]

    def as_int(self):
        if self.token != TK_INT:
            return None
        t = self.raw()  # strconv.ParseInt(s, 0, 64)
        neg = t.startswith("-")
        body = t[1:] if neg else t
        if body[:2] in ("0x", "0X"):
            v = int(body[2:], 16)
        elif len(body) > 1 and body[0] == "0":
            v = int(body[1:], 8)
        else:
            v = int(body or "0", 10)
        return -v if neg else v

    def as_float(self):
        return float(self.raw()) if self.token == TK_FLOAT else None

    def as_ident(self):
        return self.raw() if self.token == TK_IDENT else None

    def as_label(self):
        return self.raw()[:-1] if self.token == TK_LABEL else None

    def as_string(self):
        return self.raw()[1:-1].replace("\\", "") if self.token == TK_STRING else None


class _Parser:
    """read.go: function definitions, bodies, fixups; errors as `<message> @(L: l, C: c)`."""

    def __init__(self, text, program):
        self.s = _Scanner(text)
        self.p = program

    def fail(self, msg, loc=None):
        l, c = loc or self.s.lbegin
        raise ReadError("%s @(L: %d, C: %d)" % (msg, l, c))

    def unexpected(self):
        self.fail("unexpected input: '%s'" % self.s.raw())

    def next_or_fail(self):
        if not self.s.next() or self.s.token == TK_NONE:
            self.fail("unexpected end of file.")
        if self.s.token == TK_ERROR:
            self.fail("Parse error.")

    def current(self, t):
        if self.s.end():
            self.fail("unexpected end of file encountered")
        if self.s.token != t:
            self.unexpected()

    def next_token(self, t):
        self.next_or_fail()
        self.current(t)

    def skip_newlines(self):
        while self.s.token == TK_NEWLINE and self.s.next():
            pass

    def parse(self):
        while not self.s.end():
            if not self.s.next():
                break
            if self.s.token == TK_ERROR:
                self.fail("Parse error.")
            if not self.function_def():
                break

    def function_def(self):
        self.skip_newlines()
        if self.s.end():
            return False
        if self.s.token != TK_IDENT:
            self.unexpected()
        if self.s.as_ident() != "fn":
            self.fail("Expected 'fn'.")
        self.next_token(TK_IDENT)
        name = self.s.as_ident()
        self.next_token(TK_OPEN)
        params = []
        while True:
            self.next_or_fail()
            if self.s.token != TK_IDENT:
                break
            n = self.s.as_ident()
            if n not in IL.TYPES_BY_NAME:
                self.fail("Unrecognized parameter type: '%s'" % n)
            params.append(IL.TYPES_BY_NAME[n])
        self.current(TK_CLOSE)
        self.next_token(TK_IDENT)
        r = self.s.as_ident()
        if r not in IL.TYPES_BY_NAME:
            self.fail("Unrecognized return type: '%s'" % r)
        self.next_token(TK_NEWLINE)
        body = self.function_body()
        self.p.add_function(name, params, IL.TYPES_BY_NAME[r], body)
        return True

    def function_body(self):
        labels, refs, fixups, body = {}, {}, {}, []
        while True:
            self.skip_newlines()
            if self.s.token == TK_LABEL:
                labels[self.s.as_label()] = len(body)
                self.next_or_fail()
                continue
            if self.s.token != TK_IDENT:
                self.unexpected()
            word = self.s.as_ident()
            if word == "end":
                break
            if word not in IL.OP_BY_KW:
                self.fail("unrecognized opcode: '%s'" % word)
            op, args = IL.OP_BY_KW[word]
            body.append(op)
            for a in args:
                self.next_or_fail()
                if a == IL.A_STR:
                    v = self.s.as_string()
                    if v is None:
                        self.unexpected()
                    body.append(self.p.strings.add(v))
                elif a == IL.A_FN:
                    v = self.s.as_ident()
                    if v is None:
                        self.unexpected()
                    body.append(self.p.strings.add(v))
                elif a == IL.A_INT:
                    v = self.s.as_int()
                    if v is None:
                        self.unexpected()
                    body.extend(IL.int_to_words(v))
                elif a == IL.A_DBL:
                    v = self.s.as_float()
                    if v is None:
                        i = self.s.as_int()
                        if i is None:
                            self.unexpected()
                        v = float(i)
                    body.extend(IL.double_to_words(v))
                elif a == IL.A_BOOL:
                    v = self.s.as_ident()
                    if v not in ("true", "false"):
                        self.unexpected()
                    body.append(1 if v == "true" else 0)
                elif a == IL.A_ADDR:
                    v = self.s.as_ident()
                    if v is None:
                        self.unexpected()
                    fixups[len(body)] = v
                    refs[len(body)] = self.s.lbegin
                    body.append(0)
                elif a == IL.A_REG:
                    v = self.s.as_ident()
                    if v is None:
                        self.unexpected()
                    if not v.startswith("r") or not v[1:].lstrip("+-").isdigit():
                        self.fail("Invalid register name: '%s'" % v)
                    body.append(int(v[1:]) & 0xFFFFFFFF)
            self.next_token(TK_NEWLINE)
        for at, label in fixups.items():
            if label not in labels:
                self.fail("Label not found: %s" % label, refs[at])
            body[at] = labels[label]
        return body


def merge_text(text, program):
    """text.MergeText: parse `text` and add its functions to `program` (raises ReadError)."""
    _Parser(text, program).parse()
    return program


def read_text(text):
    """text.ReadText."""
    return merge_text(text, IL.Program())
