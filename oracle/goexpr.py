"""ORACLE (test infrastructure only) -- CPU restatement of Mixer's expression front end.

Restates, for parity checking:
  * the Go 1.9 ``go/scanner`` + ``go/parser.ParseExpr`` subset that ``expr.Parse`` relies on
    (mixer/pkg/expr/expr.go:424-436), including the error texts of the golden rows
    (``1:3: expected '==', found '='``, ``1:1: illegal character U+0040 '@'``);
  * ``process`` / ``flattenSelectors`` / ``generateVarName`` / ``newConstant``
    (mixer/pkg/expr/expr.go:123-152, 270-421) and the ``tMap`` operator names (expr.go:34-69);
  * ``Expression.EvalType`` / ``Function.EvalType`` (expr.go:93-105, 202-268), the intrinsic table
    (mixer/pkg/expr/func.go:39-72) and the extern metadata (mixer/pkg/il/runtime/externs.go:42-79);
  * the Go stdlib pieces the path calls: ``strconv.ParseInt(s,10,64)``, ``strconv.ParseFloat``,
    ``strconv.Unquote`` and ``time.ParseDuration`` (Go 1.9 algorithm).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use this
module, and only as the checker.  The product path (istio_amd) has its own C++ front end.
"""
from __future__ import annotations

import struct
import unicodedata

# ----------------------------------------------------------------------------------------------
# ValueType enum of istio.io/api mixer/v1/config/descriptor (rev 58de5731, Gopkg.lock:1045-1057)
VALUE_TYPES = ["VALUE_TYPE_UNSPECIFIED", "STRING", "INT64", "DOUBLE", "BOOL", "TIMESTAMP",
               "IP_ADDRESS", "EMAIL_ADDRESS", "URI", "DNS_NAME", "DURATION", "STRING_MAP"]
VT = {n: i for i, n in enumerate(VALUE_TYPES)}
UNSPEC, STRING, INT64, DOUBLE, BOOL, TIMESTAMP, IP_ADDRESS, EMAIL_ADDRESS, URI, DNS_NAME, DURATION, \
    STRING_MAP = range(12)


def vt_name(v):
    return VALUE_TYPES[v] if 0 <= v < len(VALUE_TYPES) else str(v)


class ParseError(Exception):
    pass


class TypeCheckError(Exception):
    pass


# ----------------------------------------------------------------------------------------------
# go/token
_KEYWORDS = {"break", "case", "chan", "const", "continue", "default", "defer", "else", "fallthrough",
             "for", "func", "go", "goto", "if", "import", "interface", "map", "package", "range",
             "return", "select", "struct", "switch", "type", "var"}

_OPS = ["<<=", ">>=", "&^=", "...", "&&", "||", "<-", "++", "--", "==", "!=", "<=", ">=", ":=",
        "+=", "-=", "*=", "/=", "%=", "&=", "|=", "^=", "<<", ">>", "&^",
        "+", "-", "*", "/", "%", "&", "|", "^", "<", ">", "=", "!", "(", "[", "{", ",", ".", ")",
        "]", "}", ";", ":"]

_PREC = {"||": 1, "&&": 2, "==": 3, "!=": 3, "<": 3, "<=": 3, ">": 3, ">=": 3,
         "+": 4, "-": 4, "|": 4, "^": 4, "*": 5, "/": 5, "%": 5, "<<": 5, ">>": 5, "&": 5, "&^": 5}

# expr.go:34-69
_TMAP = {"+": "ADD", "-": "SUB", "*": "MUL", "/": "QUO", "%": "REM", "&": "AND", "|": "OR",
         "^": "XOR", "&&": "LAND", "||": "LOR", "==": "EQ", "<": "LT", ">": "GT", "!": "NOT",
         "!=": "NEQ", "<=": "LEQ", ">=": "GEQ"}

_LITERAL_KINDS = ("IDENT", "INT", "FLOAT", "IMAG", "CHAR", "STRING")


class Tok:
    __slots__ = ("kind", "lit", "off")

    def __init__(self, kind, lit, off):
        self.kind = kind  # IDENT INT FLOAT IMAG CHAR STRING OP EOF ILLEGAL SEMI
        self.lit = lit
        self.off = off

    def tokstr(self):
        if self.kind == "OP":
            return self.lit
        if self.kind == "SEMI":
            return ";"
        if self.kind == "IDENT" and self.lit in _KEYWORDS:
            return self.lit
        return self.kind


def _is_letter(ch):
    return ch == "_" or ("a" <= ch <= "z") or ("A" <= ch <= "Z") or (ord(ch) >= 0x80 and ch.isalpha())


def _is_digit(ch):
    return ("0" <= ch <= "9") or (ord(ch) >= 0x80 and unicodedata.category(ch) == "Nd")


class Scanner:
    """go/scanner restricted to one source line set; offsets are byte offsets."""

    def __init__(self, src: str, errors):
        self.b = src.encode("utf-8")
        self.src = src
        self.pos = 0
        self.insert_semi = False
        self.errors = errors

    def _col(self, off):
        line = self.b.count(b"\n", 0, off) + 1
        start = self.b.rfind(b"\n", 0, off) + 1
        return line, off - start + 1

    def error(self, off, msg):
        line, col = self._col(off)
        self.errors.append((line, col, msg))

    def _ch(self, p=None):
        p = self.pos if p is None else p
        if p >= len(self.b):
            return ""
        c = self.b[p]
        if c < 0x80:
            return chr(c)
        # decode one utf-8 rune
        for n in (2, 3, 4):
            try:
                return self.b[p:p + n].decode("utf-8")
            except UnicodeDecodeError:
                continue
        return "�"

    def _adv(self):
        ch = self._ch()
        self.pos += len(ch.encode("utf-8")) if ch not in ("", "�") else 1
        return ch

    def scan(self) -> Tok:
        # skip whitespace (newline only when not inserting a semicolon)
        while True:
            ch = self._ch()
            if ch in (" ", "\t", "\r") or (ch == "\n" and not self.insert_semi):
                self.pos += 1
                continue
            break
        off = self.pos
        ch = self._ch()
        insert = False
        if ch == "":
            if self.insert_semi:
                self.insert_semi = False
                return Tok("SEMI", "\n", off)
            return Tok("EOF", "", off)
        if _is_letter(ch):
            while True:
                c = self._ch()
                if c and (_is_letter(c) or _is_digit(c)):
                    self._adv()
                else:
                    break
            lit = self.b[off:self.pos].decode("utf-8")
            insert = lit not in _KEYWORDS or lit in ("break", "continue", "fallthrough", "return")
            self.insert_semi = insert
            return Tok("IDENT", lit, off)
        if "0" <= ch <= "9" or (ch == "." and "0" <= self._ch(self.pos + 1) <= "9"):
            self.insert_semi = True
            return self._scan_number(off)
        self._adv()
        if ch == "\n":
            self.insert_semi = False
            return Tok("SEMI", "\n", off)
        if ch == '"':
            self.insert_semi = True
            return self._scan_string(off)
        if ch == "`":
            self.insert_semi = True
            while True:
                c = self._ch()
                if c == "":
                    self.error(off, "raw string literal not terminated")
                    break
                self._adv()
                if c == "`":
                    break
            return Tok("STRING", self.b[off:self.pos].decode("utf-8", "replace"), off)
        if ch == "'":
            self.insert_semi = True
            return self._scan_rune(off)
        if ch == "/" and self._ch() in ("/", "*"):
            # comments: treat as whitespace (newline handling approximated)
            if self._ch() == "/":
                while self._ch() not in ("", "\n"):
                    self._adv()
            else:
                self._adv()
                while True:
                    c = self._adv()
                    if c == "":
                        self.error(off, "comment not terminated")
                        break
                    if c == "*" and self._ch() == "/":
                        self._adv()
                        break
            return self.scan()
        # operators
        rest = self.b[off:off + 3].decode("utf-8", "replace")
        for op in _OPS:
            if rest.startswith(op):
                self.pos = off + len(op)
                self.insert_semi = op in (")", "]", "}", "++", "--")
                return Tok("OP", op, off)
        self.insert_semi = self.insert_semi  # unchanged for illegal chars
        self.error(off, "illegal character U+%04X '%s'" % (ord(ch), ch))
        return Tok("ILLEGAL", ch, off)

    def _digits(self, base):
        while True:
            c = self._ch()
            if c and ((base == 16 and c in "0123456789abcdefABCDEF") or (base != 16 and "0" <= c <= "9")):
                self.pos += 1
            else:
                break

    def _scan_number(self, off):
        kind = "INT"
        seen_point = False
        if self._ch() == ".":
            seen_point = True
        if not seen_point and self._ch() == "0":
            self.pos += 1
            if self._ch() in ("x", "X"):
                self.pos += 1
                start = self.pos
                self._digits(16)
                if self.pos == start:
                    self.error(off, "illegal hexadecimal number")
                return Tok("INT", self.b[off:self.pos].decode(), off)
            # octal or float
            seen_decimal_digit = False
            while True:
                c = self._ch()
                if c and "0" <= c <= "7":
                    self.pos += 1
                elif c in ("8", "9"):
                    seen_decimal_digit = True
                    self.pos += 1
                else:
                    break
            c = self._ch()
            if c not in (".", "e", "E", "i"):
                if seen_decimal_digit:
                    self.error(off, "illegal octal number")
                return Tok("INT", self.b[off:self.pos].decode(), off)
        else:
            if not seen_point:
                self._digits(10)
        if self._ch() == ".":
            kind = "FLOAT"
            self.pos += 1
            self._digits(10)
        if self._ch() in ("e", "E"):
            kind = "FLOAT"
            self.pos += 1
            if self._ch() in ("-", "+"):
                self.pos += 1
            start = self.pos
            self._digits(10)
            if start == self.pos:
                self.error(off, "illegal floating-point exponent")
        if self._ch() == "i":
            kind = "IMAG"
            self.pos += 1
        return Tok(kind, self.b[off:self.pos].decode(), off)

    def _scan_escape(self, quote):
        off = self.pos
        c = self._ch()
        if c in ("a", "b", "f", "n", "r", "t", "v", "\\", quote):
            self._adv()
            return True
        if c in "01234567" and c:
            n, base, mx = 3, 8, 255
        elif c == "x":
            self._adv()
            n, base, mx = 2, 16, 255
        elif c == "u":
            self._adv()
            n, base, mx = 4, 16, 0x10FFFF
        elif c == "U":
            self._adv()
            n, base, mx = 8, 16, 0x10FFFF
        else:
            msg = "unknown escape sequence"
            if c == "":
                msg = "escape sequence not terminated"
            self.error(off, msg)
            return False
        x = 0
        for _ in range(n):
            c = self._ch()
            d = int(c, 16) if c and c in "0123456789abcdefABCDEF" else 99
            if d >= base:
                msg = "illegal character %s in escape sequence" % ("U+%04X" % ord(c) if c else "EOF")
                if c == "":
                    msg = "escape sequence not terminated"
                self.error(self.pos, msg)
                return False
            x = x * base + d
            self._adv()
        if x > mx or 0xD800 <= x < 0xE000:
            self.error(off, "escape sequence is invalid Unicode code point")
            return False
        return True

    def _scan_string(self, off):
        while True:
            c = self._ch()
            if c == "\n" or c == "":
                self.error(off, "string literal not terminated")
                break
            self._adv()
            if c == '"':
                break
            if c == "\\":
                self._scan_escape('"')
        return Tok("STRING", self.b[off:self.pos].decode("utf-8", "replace"), off)

    def _scan_rune(self, off):
        valid = True
        n = 0
        while True:
            c = self._ch()
            if c == "\n" or c == "":
                if valid:
                    self.error(off, "rune literal not terminated")
                    valid = False
                break
            self._adv()
            if c == "'":
                break
            n += 1
            if c == "\\":
                if not self._scan_escape("'"):
                    valid = False
        if valid and n != 1:
            self.error(off, "illegal rune literal")
        return Tok("CHAR", self.b[off:self.pos].decode("utf-8", "replace"), off)


# ----------------------------------------------------------------------------------------------
# go/ast subset (tuples):
#   ("Ident", name) ("BasicLit", kind, value) ("Paren", x) ("Selector", x, name) ("Index", x, idx)
#   ("Call", fun, [args]) ("Unary", op, x) ("Binary", op, x, y) ("Star", x) ("Other", desc)


class _Bailout(Exception):
    pass


class GoExprParser:
    def __init__(self, src):
        self.errors = []
        self.sc = Scanner(src, self.errors)
        self.expr_lev = 0
        self.tok = None
        self.next()

    def next(self):
        self.tok = self.sc.scan()

    def error(self, off, msg):
        line, col = self.sc._col(off)
        # go/parser (Go 1.9) keeps only the first parser error on a line unless AllErrors is set.
        if self.errors and self.errors[-1][0] == line:
            return
        self.errors.append((line, col, msg))

    def error_expected(self, off, what):
        msg = "expected " + what
        if off == self.tok.off:
            if self.tok.kind == "SEMI" and self.tok.lit == "\n":
                msg += ", found newline"
            else:
                msg += ", found '" + self.tok.tokstr() + "'"
                if self.tok.kind in _LITERAL_KINDS and self.tok.tokstr() == self.tok.kind:
                    msg += " " + self.tok.lit
        self.error(off, msg)

    def expect(self, lit):
        off = self.tok.off
        if not (self.tok.kind == "OP" and self.tok.lit == lit):
            self.error_expected(off, "'" + lit + "'")
            raise _Bailout()
        self.next()
        return off

    def tok_prec(self):
        t = self.tok
        if t.kind != "OP":
            return None, 0
        op = t.lit
        if op == "=":  # parser.inRhs && tok == ASSIGN -> treated as EQL
            op = "=="
        return op, _PREC.get(op, 0)

    def parse_expr(self):
        return self.parse_binary(1)

    def parse_binary(self, prec1):
        x = self.parse_unary()
        while True:
            op, oprec = self.tok_prec()
            if oprec < prec1:
                return x
            self.expect(op)
            y = self.parse_binary(oprec + 1)
            x = ("Binary", op, x, y)

    def parse_unary(self):
        t = self.tok
        if t.kind == "OP" and t.lit in ("+", "-", "!", "^", "&"):
            self.next()
            x = self.parse_unary()
            return ("Unary", t.lit, x)
        if t.kind == "OP" and t.lit == "<-":
            self.next()
            x = self.parse_unary()
            return ("Unary", "<-", x)
        if t.kind == "OP" and t.lit == "*":
            self.next()
            x = self.parse_unary()
            return ("Star", x)
        return self.parse_primary()

    def parse_operand(self):
        t = self.tok
        if t.kind == "IDENT" and t.lit not in _KEYWORDS:
            self.next()
            return ("Ident", t.lit)
        if t.kind in ("INT", "FLOAT", "IMAG", "CHAR", "STRING"):
            self.next()
            return ("BasicLit", t.kind, t.lit)
        if t.kind == "OP" and t.lit == "(":
            self.next()
            self.expr_lev += 1
            x = self.parse_expr_or_type()
            self.expr_lev -= 1
            self.expect(")")
            return ("Paren", x)
        typ = self.try_type()
        if typ is not None:
            return typ
        self.error_expected(t.off, "operand")
        raise _Bailout()

    def try_type(self):
        """Types that may start an operand (composite literal / conversion)."""
        t = self.tok
        if t.kind == "OP" and t.lit == "[":
            self.next()
            depth = 1
            while depth:
                if self.tok.kind == "EOF":
                    self.error_expected(self.tok.off, "']'")
                    raise _Bailout()
                if self.tok.kind == "OP" and self.tok.lit == "[":
                    depth += 1
                if self.tok.kind == "OP" and self.tok.lit == "]":
                    depth -= 1
                self.next()
            self.parse_type_rest()
            return ("Other", "ArrayType")
        if t.kind == "IDENT" and t.lit in ("map", "chan", "struct", "interface", "func"):
            self.next()
            self.parse_type_rest(t.lit)
            return ("Other", t.lit)
        return None

    def parse_type_rest(self, kw=None):
        # Consume a (simplified) type suffix: brackets/braces/parens balanced, or an identifier chain.
        if kw in ("struct", "interface"):
            if self.tok.kind == "OP" and self.tok.lit == "{":
                self._skip_balanced("{", "}")
            return
        if kw == "func":
            if self.tok.kind == "OP" and self.tok.lit == "(":
                self._skip_balanced("(", ")")
            if self.tok.kind == "OP" and self.tok.lit == "{":
                self._skip_balanced("{", "}")
            return
        if kw == "map":
            if self.tok.kind == "OP" and self.tok.lit == "[":
                self._skip_balanced("[", "]")
        if self.tok.kind == "IDENT":
            self.next()
            while self.tok.kind == "OP" and self.tok.lit == ".":
                self.next()
                if self.tok.kind == "IDENT":
                    self.next()
        elif self.tok.kind == "OP" and self.tok.lit == "*":
            self.next()
            self.parse_type_rest()
        elif self.tok.kind == "OP" and self.tok.lit == "[":
            self.try_type()

    def _skip_balanced(self, o, c):
        depth = 0
        while True:
            if self.tok.kind == "EOF":
                self.error_expected(self.tok.off, "'" + c + "'")
                raise _Bailout()
            if self.tok.kind == "OP" and self.tok.lit == o:
                depth += 1
            if self.tok.kind == "OP" and self.tok.lit == c:
                depth -= 1
                if depth == 0:
                    self.next()
                    return
            self.next()

    def parse_expr_or_type(self):
        return self.parse_expr()

    @staticmethod
    def _is_literal_type(x):
        if x[0] == "Ident":
            return True
        if x[0] == "Selector":
            return x[1][0] == "Ident"
        if x[0] == "Other" and x[1] in ("ArrayType", "map", "struct"):
            return True
        return False

    def parse_primary(self):
        x = self.parse_operand()
        while True:
            t = self.tok
            if t.kind == "OP" and t.lit == ".":
                self.next()
                if self.tok.kind == "IDENT":
                    name = self.tok.lit
                    self.next()
                    x = ("Selector", x, name)
                elif self.tok.kind == "OP" and self.tok.lit == "(":
                    self.next()
                    if self.tok.kind == "IDENT" and self.tok.lit == "type":
                        self.next()
                    else:
                        self.parse_expr_or_type()
                    self.expect(")")
                    x = ("Other", "TypeAssertExpr")
                else:
                    self.error_expected(self.tok.off, "selector or type assertion")
                    raise _Bailout()
            elif t.kind == "OP" and t.lit == "[":
                self.next()
                self.expr_lev += 1
                idx = [None, None, None]
                ncolons = 0
                if not (self.tok.kind == "OP" and self.tok.lit == ":"):
                    idx[0] = self.parse_expr()
                while self.tok.kind == "OP" and self.tok.lit == ":" and ncolons < 2:
                    ncolons += 1
                    self.next()
                    if not (self.tok.kind == "OP" and self.tok.lit in (":", "]")):
                        idx[ncolons] = self.parse_expr()
                self.expr_lev -= 1
                self.expect("]")
                if ncolons > 0:
                    x = ("Other", "SliceExpr")
                else:
                    x = ("Index", x, idx[0])
            elif t.kind == "OP" and t.lit == "(":
                self.next()
                self.expr_lev += 1
                args = []
                while not (self.tok.kind == "OP" and self.tok.lit == ")") and self.tok.kind != "EOF":
                    args.append(self.parse_expr_or_type())
                    if self.tok.kind == "OP" and self.tok.lit == "...":
                        self.next()
                    if not (self.tok.kind == "OP" and self.tok.lit == ","):
                        break
                    self.next()
                self.expr_lev -= 1
                self.expect(")")
                x = ("Call", x, args)
            elif t.kind == "OP" and t.lit == "{":
                if self._is_literal_type(x) and (self.expr_lev >= 0 or x[0] not in ("Ident", "Selector")):
                    self._skip_balanced("{", "}")
                    x = ("Other", "CompositeLit")
                else:
                    return x
            else:
                return x

    def parse(self):
        try:
            x = self.parse_expr()
            if self.tok.kind == "SEMI" and self.tok.lit == "\n":
                self.next()
            if self.tok.kind != "EOF":
                self.error_expected(self.tok.off, "'EOF'")
                raise _Bailout()
        except _Bailout:
            x = None
            # drain the scanner so later scanner errors are still recorded
            while self.tok.kind != "EOF":
                self.next()
        if self.errors:
            errs = sorted(self.errors, key=lambda e: (e[0], e[1]))
            first = "%d:%d: %s" % errs[0]
            if len(errs) > 1:
                first = "%s (and %d more errors)" % (first, len(errs) - 1)
            raise ParseError(first)
        return x


# ----------------------------------------------------------------------------------------------
# strconv / time restatements (Go 1.9)

def go_unquote(s: str):
    """strconv.Unquote. Returns str or raises ValueError('invalid syntax')."""
    if len(s) < 2:
        raise ValueError("invalid syntax")
    q = s[0]
    if q != s[-1]:
        raise ValueError("invalid syntax")
    body = s[1:-1]
    if q == "`":
        if "`" in body:
            raise ValueError("invalid syntax")
        return body.replace("\r", "")
    if q not in ('"', "'"):
        raise ValueError("invalid syntax")
    if "\n" in body:
        raise ValueError("invalid syntax")
    if "\\" not in body and q not in body:
        if q == '"':
            return body
        if q == "'" and len(body) == 1:
            return body
    out = []
    i = 0
    b = body
    while i < len(b):
        c = b[i]
        if c == q and q == "'":
            raise ValueError("invalid syntax")
        if c == q:
            raise ValueError("invalid syntax")
        if c != "\\":
            out.append(c)
            i += 1
        else:
            i += 1
            if i >= len(b):
                raise ValueError("invalid syntax")
            e = b[i]
            i += 1
            simple = {"a": "\a", "b": "\b", "f": "\f", "n": "\n", "r": "\r", "t": "\t", "v": "\v",
                      "\\": "\\"}
            if e in simple:
                out.append(simple[e])
            elif e in ("'", '"'):
                if e != q:
                    raise ValueError("invalid syntax")
                out.append(e)
            elif e in ("x", "u", "U"):
                n = {"x": 2, "u": 4, "U": 8}[e]
                h = b[i:i + n]
                if len(h) < n or any(ch not in "0123456789abcdefABCDEF" for ch in h):
                    raise ValueError("invalid syntax")
                v = int(h, 16)
                i += n
                if e == "x":
                    out.append(chr(0xDC00 + v) if v >= 0x80 else chr(v))  # raw byte (surrogateescape)
                else:
                    if v > 0x10FFFF or 0xD800 <= v < 0xE000:
                        raise ValueError("invalid syntax")
                    out.append(chr(v))
            elif e in "01234567":
                h = b[i - 1:i + 2]
                if len(h) < 3 or any(ch not in "01234567" for ch in h):
                    raise ValueError("invalid syntax")
                v = int(h, 8)
                if v > 255:
                    raise ValueError("invalid syntax")
                i += 2
                out.append(chr(0xDC00 + v) if v >= 0x80 else chr(v))  # raw byte (surrogateescape)
            else:
                raise ValueError("invalid syntax")
        if q == "'" and len(out) > 1:
            raise ValueError("invalid syntax")
    res = "".join(out)
    if q == "'" and len(out) != 1:
        raise ValueError("invalid syntax")
    return res


_MAX_I64 = (1 << 63) - 1
_UNITS = {b"ns": 1, b"us": 1000, "µs".encode(): 1000, "μs".encode(): 1000, b"ms": 1000000,
          b"s": 1000000000, b"m": 60 * 1000000000, b"h": 3600 * 1000000000}


def _to_i64(v):
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >> 63 else v


def go_parse_duration(text: str) -> int:
    """time.ParseDuration (Go 1.9). Raises ValueError with Go's message."""
    orig = text
    s = text.encode("utf-8")
    d = 0
    neg = False
    if s:
        c = s[0:1]
        if c in (b"-", b"+"):
            neg = c == b"-"
            s = s[1:]
    if s == b"0":
        return 0
    if not s:
        raise ValueError("time: invalid duration " + orig)
    while s:
        f = 0
        scale = 1.0
        if not (s[0:1] == b"." or b"0" <= s[0:1] <= b"9"):
            raise ValueError("time: invalid duration " + orig)
        pl = len(s)
        # leadingInt
        v = 0
        i = 0
        while i < len(s) and 0x30 <= s[i] <= 0x39:
            if v > _MAX_I64 // 10:
                raise ValueError("time: invalid duration " + orig)
            v = v * 10 + s[i] - 0x30
            if v > _MAX_I64:
                raise ValueError("time: invalid duration " + orig)
            i += 1
        s = s[i:]
        pre = pl != len(s)
        post = False
        if s and s[0:1] == b".":
            s = s[1:]
            pl2 = len(s)
            i = 0
            overflow = False
            while i < len(s) and 0x30 <= s[i] <= 0x39:
                if not overflow:
                    if f > _MAX_I64 // 10:
                        overflow = True
                    else:
                        y = f * 10 + s[i] - 0x30
                        if y > _MAX_I64:
                            overflow = True
                        else:
                            f = y
                            scale *= 10
                i += 1
            s = s[i:]
            post = pl2 != len(s)
        if not pre and not post:
            raise ValueError("time: invalid duration " + orig)
        i = 0
        while i < len(s) and not (s[i] == 0x2E or 0x30 <= s[i] <= 0x39):
            i += 1
        if i == 0:
            raise ValueError("time: missing unit in duration " + orig)
        u = s[:i]
        s = s[i:]
        if u not in _UNITS:
            raise ValueError("time: unknown unit " + u.decode("utf-8", "replace") + " in duration " + orig)
        unit = _UNITS[u]
        if v > _MAX_I64 // unit:
            raise ValueError("time: invalid duration " + orig)
        v *= unit
        if f > 0:
            add = float(f) * (float(unit) / scale)
            v = _to_i64(v + int(add))
            if v < 0:
                raise ValueError("time: invalid duration " + orig)
        d = _to_i64(d + v)
        if d < 0:
            raise ValueError("time: invalid duration " + orig)
    if neg:
        d = -d
    return d


def go_parse_int10(s: str) -> int:
    """strconv.ParseInt(s, 10, 64)."""
    fn = "strconv.ParseInt"
    if not s:
        raise ValueError('%s: parsing "%s": invalid syntax' % (fn, s))
    body = s
    if body[0] in "+-":
        body = body[1:]
    if not body or any(c not in "0123456789" for c in body):
        raise ValueError('%s: parsing "%s": invalid syntax' % (fn, s))
    v = int(s, 10)
    if v > _MAX_I64 or v < -_MAX_I64 - 1:
        raise ValueError('%s: parsing "%s": value out of range' % (fn, s))
    return v


def go_parse_float(s: str) -> float:
    """strconv.ParseFloat(s, 64) for Go FLOAT tokens."""
    try:
        v = float(s)
    except ValueError:
        raise ValueError('strconv.ParseFloat: parsing "%s": invalid syntax' % s)
    if v in (float("inf"), float("-inf")) and "inf" not in s.lower():
        raise ValueError('strconv.ParseFloat: parsing "%s": value out of range' % s)
    return v


# ----------------------------------------------------------------------------------------------
# mixer/pkg/expr AST (expr.go:78-199)

class Constant:
    __slots__ = ("str_value", "value", "type")

    def __init__(self, str_value, value, typ):
        self.str_value = str_value
        self.value = value
        self.type = typ

    def __str__(self):
        return self.str_value


class Variable:
    __slots__ = ("name",)

    def __init__(self, name):
        self.name = name

    def __str__(self):
        return "$" + self.name


class Function:
    __slots__ = ("name", "target", "args")

    def __init__(self, name, target=None, args=None):
        self.name = name
        self.target = target
        self.args = args or []

    def __str__(self):
        s = ""
        if self.target is not None:
            s += str(self.target) + ":"
        s += self.name + "(" + ", ".join(str(a) for a in self.args) + ")"
        return s


class Expression:
    __slots__ = ("const", "var", "fn")

    def __init__(self):
        self.const = None
        self.var = None
        self.fn = None

    def __str__(self):
        if self.const is not None:
            return str(self.const)
        if self.var is not None:
            return str(self.var)
        if self.fn is not None:
            return str(self.fn)
        return "<nil>"


class Duration(int):
    """time.Duration constant value (an int64 of nanoseconds)."""


_TYPEMAP = {"INT": INT64, "FLOAT": DOUBLE, "CHAR": STRING, "STRING": STRING}  # expr.go:71-76


def new_constant(v: str, vtype: int) -> Constant:
    """expr.go:123-152."""
    if vtype == INT64:
        return Constant(v, go_parse_int10(v), vtype)
    if vtype == DOUBLE:
        return Constant(v, go_parse_float(v), vtype)
    try:
        unq = go_unquote(v)
    except ValueError:
        raise ParseError("invalid syntax")
    try:
        d = go_parse_duration(unq)
        return Constant(v, Duration(d), DURATION)
    except ValueError:
        pass
    return Constant(v, unq, vtype)


def _unexpected(node):
    return ParseError("unexpected expression: %s" % (node,))


def _generate_var_name(selectors):
    """expr.go:270-285."""
    return ".".join(reversed(selectors))


def _flatten_selectors(sel):
    """expr.go:384-408. Returns (anchor, parts)."""
    parts = []
    ex = sel
    while True:
        parts.append(ex[2])
        x = ex[1]
        if x[0] == "Selector":
            ex = x
        elif x[0] == "Ident":
            parts.append(x[1])
            return None, parts
        elif x[0] in ("Call", "BasicLit", "Paren"):
            return x, parts
        else:
            raise _unexpected(x)


def _process(node, tgt: Expression):
    """expr.go:287-382."""
    k = node[0]
    if k == "Unary":
        tgt.fn = Function(_TMAP.get(node[1], ""))
        _process_func(tgt.fn, [node[2]])
    elif k == "Binary":
        tgt.fn = Function(_TMAP.get(node[1], ""))
        _process_func(tgt.fn, [node[2], node[3]])
    elif k == "Call":
        fun = node[1]
        if fun[0] == "Selector":
            anchor, w = _flatten_selectors(fun)
            if anchor is None:
                inst = Expression()
                inst.var = Variable(_generate_var_name(w[1:]))
                tgt.fn = Function(w[0], target=inst)
            else:
                afn = Expression()
                _process(anchor, afn)
                if len(w) != 1:
                    raise _unexpected(fun)
                tgt.fn = Function(w[0], target=afn)
            _process_func(tgt.fn, node[2])
        elif fun[0] == "Ident":
            tgt.fn = Function(fun[1])
            _process_func(tgt.fn, node[2])
        else:
            # The reference leaves tgt empty here (its inner type switch has no default): a later
            # EvalType dereferences a nil Fn and panics.
            pass
    elif k == "Paren":
        _process(node[1], tgt)
    elif k == "BasicLit":
        try:
            tgt.const = new_constant(node[2], _TYPEMAP.get(node[1], UNSPEC))
        except ParseError:
            raise
        except ValueError as e:
            raise ParseError(str(e))
    elif k == "Ident":
        lv = node[1].lower()
        if lv in ("true", "false"):
            tgt.const = Constant(lv, lv == "true", BOOL)
        else:
            tgt.var = Variable(node[1])
    elif k == "Selector":
        anchor, w = _flatten_selectors(node)
        if anchor is not None:
            raise _unexpected(node)
        tgt.var = Variable(_generate_var_name(w))
    elif k == "Index":
        tgt.fn = Function("INDEX")
        _process_func(tgt.fn, [node[1], node[2]])
    else:
        raise _unexpected(node)


def _process_func(fn, args):
    fn.args = []
    for a in args:
        e = Expression()
        fn.args.append(e)
        _process(a, e)


def parse(src: str) -> Expression:
    """expr.Parse (expr.go:424-436)."""
    try:
        ast = GoExprParser(src).parse()
    except ParseError as e:
        raise ParseError("unable to parse expression '%s': %s" % (src, e))
    ex = Expression()
    _process(ast, ex)
    return ex


# ----------------------------------------------------------------------------------------------
# Function metadata (func.go:21-85, il/runtime/externs.go:42-79)

class FunctionMetadata:
    __slots__ = ("name", "instance", "target_type", "return_type", "argument_types")

    def __init__(self, name, instance=False, target_type=UNSPEC, return_type=UNSPEC, argument_types=()):
        self.name = name
        self.instance = instance
        self.target_type = target_type
        self.return_type = return_type
        self.argument_types = list(argument_types)


def intrinsics():
    return [
        FunctionMetadata("EQ", return_type=BOOL, argument_types=[UNSPEC, UNSPEC]),
        FunctionMetadata("NEQ", return_type=BOOL, argument_types=[UNSPEC, UNSPEC]),
        FunctionMetadata("OR", return_type=UNSPEC, argument_types=[UNSPEC, UNSPEC]),
        FunctionMetadata("LOR", return_type=BOOL, argument_types=[BOOL, BOOL]),
        FunctionMetadata("LAND", return_type=BOOL, argument_types=[BOOL, BOOL]),
        FunctionMetadata("INDEX", return_type=STRING, argument_types=[STRING_MAP, STRING]),
    ]


def extern_metadata():
    return [
        FunctionMetadata("ip", return_type=IP_ADDRESS, argument_types=[STRING]),
        FunctionMetadata("timestamp", return_type=TIMESTAMP, argument_types=[STRING]),
        FunctionMetadata("match", return_type=BOOL, argument_types=[STRING, STRING]),
        FunctionMetadata("matches", instance=True, target_type=STRING, return_type=BOOL, argument_types=[STRING]),
        FunctionMetadata("startsWith", instance=True, target_type=STRING, return_type=BOOL, argument_types=[STRING]),
        FunctionMetadata("endsWith", instance=True, target_type=STRING, return_type=BOOL, argument_types=[STRING]),
    ]


def func_map(functions=None):
    m = {}
    for f in intrinsics():
        m[f.name] = f
    for f in (extern_metadata() if functions is None else functions):
        m[f.name] = f
    return m


class EvalPanic(Exception):
    """A Go runtime panic in the reference (e.g. nil Fn dereference)."""


def eval_type(e: Expression, attrs: dict, fmap: dict) -> int:
    """Expression.EvalType (expr.go:93-105). attrs: name -> ValueType int."""
    if e.const is not None:
        return e.const.type
    if e.var is not None:
        if e.var.name not in attrs:
            raise TypeCheckError("unknown attribute %s" % e.var.name)
        return attrs[e.var.name]
    if e.fn is None:
        raise EvalPanic("runtime error: invalid memory address or nil pointer dereference")
    return fn_eval_type(e.fn, attrs, fmap)


def fn_eval_type(f: Function, attrs, fmap) -> int:
    """Function.EvalType (expr.go:202-268)."""
    fn = fmap.get(f.name)
    if fn is None:
        raise TypeCheckError("unknown function: %s" % f.name)
    tmpl = UNSPEC
    if f.target is not None:
        if not fn.instance:
            raise TypeCheckError("invoking regular function on instance method: %s" % f.name)
        tt = eval_type(f.target, attrs, fmap)
        if fn.target_type == UNSPEC:
            tmpl = tt
        elif tt != fn.target_type:
            raise TypeCheckError("%s target typeError got %s, expected %s" % (f, vt_name(tt), vt_name(fn.target_type)))
    elif fn.instance:
        raise TypeCheckError("invoking instance method without an instance: %s" % f.name)
    argtypes = fn.argument_types
    if len(f.args) < len(argtypes):
        raise TypeCheckError("%s arity mismatch. Got %d arg(s), expected %d arg(s)" % (f, len(f.args), len(argtypes)))
    for idx in range(min(len(f.args), len(argtypes))):
        at = eval_type(f.args[idx], attrs, fmap)
        exp = argtypes[idx]
        if exp == UNSPEC:
            if tmpl == UNSPEC:
                tmpl = at
                continue
            exp = tmpl
        if at != exp:
            raise TypeCheckError("%s arg %d (%s) typeError got %s, expected %s" % (f, idx + 1, f.args[idx], vt_name(at), vt_name(exp)))
    ret = fn.return_type
    if ret == UNSPEC:
        ret = tmpl
    return ret


def extract_eq_matches(src: str) -> dict:
    """ExtractEQMatches (expr.go:446-490)."""
    ex = parse(src)
    out = {}

    def rec(e):
        if e.fn is None:
            return
        f = e.fn
        if f.name == "EQ":
            if f.args[0].var is not None and f.args[1].const is not None:
                out[f.args[0].var.name] = f.args[1].const.value
            elif f.args[0].const is not None and f.args[1].var is not None:
                out[f.args[1].var.name] = f.args[0].const.value
        if f.name != "LAND":
            return
        for a in f.args:
            rec(a)

    rec(ex)
    return out


def float_bits(d: float):
    """(low word, high word) of math.Float64bits (il/convert.go:31-35)."""
    u = struct.unpack("<Q", struct.pack("<d", d))[0]
    return u & 0xFFFFFFFF, u >> 32
