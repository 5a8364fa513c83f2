"""Minimal Go-source reader used ONLY to turn the reference's Go test tables into JSON fixtures.

It understands the subset of Go composite-literal syntax the reference's table-driven tests use:
string / raw-string / rune / number literals, identifiers and selectors, calls such as
``int64(..)`` / ``[]uint8(net.ParseIP(..))``, ``+`` concatenation, and composite literals
``T{k: v, ...}`` with or without an explicit type.  Function literals (``func(..) {..}``) are kept as
opaque ``("func", src)`` nodes.  Nothing from the reference is executed; the fixtures are data.
"""
from __future__ import annotations

import re

_TOKEN_RE = re.compile(
    r"""
    (?P<ws>[ \t\r\n]+)
  | (?P<lcomment>//[^\n]*)
  | (?P<bcomment>/\*.*?\*/)
  | (?P<raw>`[^`]*`)
  | (?P<str>"(?:[^"\\\n]|\\.)*")
  | (?P<rune>'(?:[^'\\\n]|\\.)+')
  | (?P<num>0[xX][0-9a-fA-F]+|\d+\.\d*(?:[eE][+-]?\d+)?|\.\d+(?:[eE][+-]?\d+)?|\d+[eE][+-]?\d+|\d+)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*)
  | (?P<op>:=|\.\.\.|&&|\|\||==|!=|<=|>=|[{}()\[\],:;.+\-*/%<>=!&|^])
    """,
    re.S | re.X,
)


def tokenize(src: str):
    toks = []
    pos = 0
    while pos < len(src):
        m = _TOKEN_RE.match(src, pos)
        if not m:
            raise ValueError("cannot tokenize at %r" % src[pos:pos + 40])
        kind = m.lastgroup
        text = m.group(kind)
        if kind not in ("ws", "lcomment", "bcomment"):
            toks.append((kind, text, pos))
        pos = m.end()
    return toks


def go_unquote(lit: str) -> str:
    """strconv.Unquote for the literal forms that appear in the test tables."""
    if lit.startswith("`"):
        return lit[1:-1].replace("\r", "")
    body = lit[1:-1]
    out = []
    i = 0
    while i < len(body):
        c = body[i]
        if c != "\\":
            out.append(c)
            i += 1
            continue
        n = body[i + 1]
        simple = {"a": "\a", "b": "\b", "f": "\f", "n": "\n", "r": "\r", "t": "\t", "v": "\v",
                  "\\": "\\", "'": "'", '"': '"'}
        if n in simple:
            out.append(simple[n])
            i += 2
        elif n == "x":
            out.append(chr(int(body[i + 2:i + 4], 16)))
            i += 4
        elif n == "u":
            out.append(chr(int(body[i + 2:i + 6], 16)))
            i += 6
        elif n == "U":
            out.append(chr(int(body[i + 2:i + 10], 16)))
            i += 10
        elif n in "01234567":
            out.append(chr(int(body[i + 1:i + 4], 8)))
            i += 4
        else:
            raise ValueError("bad escape in %r" % lit)
    return "".join(out)


class Parser:
    """Recursive-descent parser over the token list producing plain Python tuples."""

    def __init__(self, src: str, start: int = 0):
        self.src = src
        self.toks = tokenize(src)
        self.i = 0
        while self.i < len(self.toks) and self.toks[self.i][2] < start:
            self.i += 1

    def peek(self, k=0):
        j = self.i + k
        return self.toks[j] if j < len(self.toks) else ("eof", "", len(self.src))

    def next(self):
        t = self.peek()
        self.i += 1
        return t

    def expect(self, text):
        t = self.next()
        if t[1] != text:
            raise ValueError("expected %r got %r near %r" % (text, t[1], self.src[t[2]:t[2] + 60]))
        return t

    # type expressions: []X, map[K]V, pkg.Name, Name, interface{}
    def parse_type(self):
        t = self.peek()
        if t[1] == "*":
            self.next()
            return "*" + self.parse_type()
        if t[1] == "[":
            self.next()
            self.expect("]")
            return "[]" + self.parse_type()
        if t[1] == "map":
            self.next()
            self.expect("[")
            k = self.parse_type()
            self.expect("]")
            return "map[%s]%s" % (k, self.parse_type())
        if t[1] == "interface":
            self.next()
            self.expect("{")
            self.expect("}")
            return "interface{}"
        name = self.next()[1]
        while self.peek()[1] == "." and self.peek(1)[0] == "ident":
            self.next()
            name += "." + self.next()[1]
        return name

    def parse_value(self):
        v = self.parse_term()
        while self.peek()[1] in ("+", "-"):
            op = self.next()[1]
            v = ("concat" if op == "+" else "sub", v, self.parse_term())
        return v

    def parse_term(self):
        v = self.parse_unary()
        while self.peek()[1] == "*":
            self.next()
            v = ("mul", v, self.parse_unary())
        return v

    def parse_unary(self):
        t = self.peek()
        if t[1] == "-":
            self.next()
            return ("neg", self.parse_unary())
        return self.parse_primary()

    def skip_balanced(self, open_, close):
        depth = 0
        start = self.peek()[2]
        while True:
            t = self.next()
            if t[1] == open_:
                depth += 1
            elif t[1] == close:
                depth -= 1
                if depth == 0:
                    return self.src[start:t[2] + 1]

    def parse_primary(self):
        t = self.peek()
        if t[0] in ("str", "raw"):
            self.next()
            return ("str", go_unquote(t[1]))
        if t[0] == "rune":
            self.next()
            return ("rune", go_unquote(t[1]))
        if t[0] == "num":
            self.next()
            return ("num", t[1])
        if t[1] == "{":
            return self.parse_composite(None)
        if t[1] == "func":
            start = t[2]
            self.next()
            self.skip_balanced("(", ")")
            # result type(s) up to the body
            while self.peek()[1] != "{":
                self.next()
            body = self.skip_balanced("{", "}")
            return ("func", self.src[start:start] + body)
        if t[1] in ("[", "map", "interface"):
            typ = self.parse_type()
            if self.peek()[1] == "{":
                return self.parse_composite(typ)
            if self.peek()[1] == "(":
                self.next()
                arg = self.parse_value()
                self.expect(")")
                return ("conv", typ, arg)
            raise ValueError("bad type expression")
        if t[0] == "ident":
            name = self.next()[1]
            while self.peek()[1] == "." and self.peek(1)[0] == "ident":
                self.next()
                name += "." + self.next()[1]
            nt = self.peek()[1]
            if nt == "(":
                self.next()
                args = []
                while self.peek()[1] != ")":
                    args.append(self.parse_value())
                    if self.peek()[1] == ",":
                        self.next()
                self.expect(")")
                return ("call", name, args)
            if nt == "{" and name[0].isupper() or (nt == "{" and "." in name and name.split(".")[-1][0].isupper()):
                return self.parse_composite(name)
            return ("ident", name)
        raise ValueError("unexpected token %r near %r" % (t[1], self.src[t[2]:t[2] + 60]))

    def parse_composite(self, typ):
        self.expect("{")
        elems = []
        while self.peek()[1] != "}":
            first = self.parse_value()
            if self.peek()[1] == ":":
                self.next()
                val = self.parse_value()
                elems.append((first, val))
            else:
                elems.append((None, first))
            if self.peek()[1] == ",":
                self.next()
        self.expect("}")
        return ("composite", typ, elems)


def find_var(src: str, name: str):
    """Return the parsed value of ``var <name> = <value>`` in src."""
    m = re.search(r"^var\s+%s\s*=\s*" % re.escape(name), src, re.M)
    if not m:
        raise KeyError(name)
    p = Parser(src, m.end())
    return p.parse_value()
