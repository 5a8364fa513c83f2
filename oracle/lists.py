"""ORACLE (test infrastructure only) -- restatement of Mixer's list adapter (mixer/adapter/list).

  HandleListEntry            list.go:68-101     code: INVALID_ARGUMENT on a check error, else
                                                 blacklist: PERMISSION_DENIED if found / whitelist:
                                                 NOT_FOUND if not found, OK otherwise
  parseStringList            stringList.go:29-47 set of non-empty lines + overrides
  parseCaseInsensitive...    stringList.go:49-67 the same after strings.ToUpper
  checkList (strings)        stringList.go:73-80 exact / ToUpper membership
  parseIPList / addEntry     ipList.go:35-75    "/32" appended without '/', net.ParseCIDR; a bad
                                                 entry fails the list, bad overrides are ignored
  checkList (IP)             ipList.go:77-92    net.ParseIP, linear IPNet.Contains scan (C, lists_oracle.c)

strings.ToUpper (Go 1.9 src/strings/strings.go: Map(unicode.ToUpper, s)) is restated rune by rune:
Go's range-loop UTF-8 decoding (an invalid byte is U+FFFD of width 1), the input's own bytes until
the first rune whose upper case differs, utf8.EncodeRune of every rune from there on (so a later
invalid byte becomes EF BF BD).  unicode.ToUpper above ASCII is the Unicode 9.0 simple uppercase
mapping of oracle/unicode_upper.json (tools/gen_oracle_upper.py: UnicodeData field 12 per code point
through Perl's charinfo, cut to runes and capitals assigned by 9.0 -- derived independently of the
engine's range table).  PARITY UNPINNED beyond the known answers in tests/test_go_upper.py: no
reference fixture has non-ASCII case-insensitive entries (list_test.go:286-342 is ASCII).
"""
from __future__ import annotations

import ctypes

import numpy as np

OK, INVALID_ARGUMENT, NOT_FOUND, PERMISSION_DENIED = 0, 3, 5, 7
STRINGS, CASE_INSENSITIVE_STRINGS, IP_ADDRESSES, REGEX = 0, 1, 2, 3


def _b(x):
    return x.encode("utf-8", "surrogateescape") if isinstance(x, str) else bytes(x)


_UPPER = None


def go_upper_rune(r: int) -> int:
    """unicode.ToUpper (Go 1.9 src/unicode/letter.go:224-232)."""
    global _UPPER
    if r < 0x80:
        return r - 32 if 0x61 <= r <= 0x7A else r
    if _UPPER is None:
        import json
        import os
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "unicode_upper.json")) as f:
            _UPPER = {a: b for a, b in json.load(f)["pairs"]}
    return _UPPER.get(r, r)


def go_decode_rune(s: bytes, i: int):
    """utf8.DecodeRuneInString(s[i:]) (Go 1.9 src/unicode/utf8/utf8.go:199-245): (rune, width);
    invalid or truncated -> (U+FFFD, 1)."""
    c0 = s[i]
    if c0 < 0x80:
        return c0, 1
    n = len(s) - i
    if 0xC2 <= c0 <= 0xDF:
        if n >= 2 and 0x80 <= s[i + 1] <= 0xBF:
            return (c0 & 0x1F) << 6 | (s[i + 1] & 0x3F), 2
    elif 0xE0 <= c0 <= 0xEF:
        lo = 0xA0 if c0 == 0xE0 else 0x80
        hi = 0x9F if c0 == 0xED else 0xBF
        if n >= 3 and lo <= s[i + 1] <= hi and 0x80 <= s[i + 2] <= 0xBF:
            return (c0 & 0x0F) << 12 | (s[i + 1] & 0x3F) << 6 | (s[i + 2] & 0x3F), 3
    elif 0xF0 <= c0 <= 0xF4:
        lo = 0x90 if c0 == 0xF0 else 0x80
        hi = 0x8F if c0 == 0xF4 else 0xBF
        if n >= 4 and lo <= s[i + 1] <= hi and 0x80 <= s[i + 2] <= 0xBF and 0x80 <= s[i + 3] <= 0xBF:
            return (c0 & 0x07) << 18 | (s[i + 1] & 0x3F) << 12 | (s[i + 2] & 0x3F) << 6 | (s[i + 3] & 0x3F), 4
    return 0xFFFD, 1


def go_to_upper(s: bytes) -> bytes:
    """strings.ToUpper = strings.Map(unicode.ToUpper, s) (Go 1.9 src/strings/strings.go:398-433,
    :541): b stays nil (the input is returned) while every rune maps to itself; at the first rune
    that changes, the bytes before it are copied as they are and every rune from it on is
    EncodeRune'd."""
    out = None
    i = 0
    while i < len(s):
        c, w = go_decode_rune(s, i)
        r = go_upper_rune(c)
        if out is None:
            if r == c:
                i += w
                continue
            out = bytearray(s[:i])
        out += chr(r).encode("utf-8", "surrogatepass")
        i += w
    return bytes(s) if out is None else bytes(out)


class StringList:
    def __init__(self, lines, overrides=(), case_insensitive=False):
        self.ci = case_insensitive
        self.entries = set()
        for s in list(lines) + list(overrides):
            s = _b(s)
            if s:
                self.entries.add(go_to_upper(s) if self.ci else s)

    def num_entries(self):
        return len(self.entries)

    def found(self, symbols):
        return np.array([1 if (go_to_upper(_b(s)) if self.ci else _b(s)) in self.entries else 0 for s in symbols],
                        dtype=np.int8)


class CStringList:
    """The same list in the C restatement (lists_oracle.c: a hash set, Go strings.ToUpper in C):
    the compiled, multi-threaded CPU baseline; tests check it against StringList."""

    def __init__(self, lines, overrides=(), case_insensitive=False):
        import oracle
        self.L = oracle.lib()
        blob, off = _blob([_b(s) for s in list(lines) + list(overrides)])
        self.h = self.L.oracle_strlist_new(blob.ctypes.data, off.ctypes.data, len(off) - 1, int(case_insensitive))

    def num_entries(self):
        return self.L.oracle_strlist_entries(self.h)

    def found(self, symbols, threads=16):
        sb, so = _blob([_b(s) for s in symbols])
        out = np.zeros(len(symbols), dtype=np.int8)
        self.L.oracle_strlist_found(self.h, sb.ctypes.data, so.ctypes.data, len(symbols), out.ctypes.data, threads)
        return out

    def __del__(self):
        try:
            self.L.oracle_strlist_free(self.h)
        except Exception:
            pass


class ListParseError(Exception):
    pass


class IPList:
    def __init__(self, whitelist, overrides=()):
        import oracle  # liboracle.so
        self.lib = oracle.lib()
        self.lib.oracle_parse_cidr.restype = ctypes.c_int
        self.lib.oracle_parse_cidr.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
        self.lib.oracle_onet_size.restype = ctypes.c_size_t
        self.size = self.lib.oracle_onet_size()
        nets = []
        for ip in whitelist:
            n = self._add(_b(ip))
            if n is None:
                orig = _b(ip).decode("utf-8", "surrogateescape")
                full = orig if "/" in orig else orig + "/32"
                raise ListParseError("could not parse list entry %s: invalid CIDR address: %s" % (orig, full))
            nets.append(n)
        for ip in overrides:
            n = self._add(_b(ip))
            if n is not None:
                nets.append(n)
        self.nets = b"".join(nets)
        self.n = len(nets)

    def _add(self, ip: bytes):
        if b"/" not in ip:
            ip += b"/32"
        buf = ctypes.create_string_buffer(self.size)
        return bytes(buf.raw) if self.lib.oracle_parse_cidr(ip, len(ip), buf) else None

    def num_entries(self):
        return self.n

    def found(self, symbols, threads=8):
        """1 found, 0 not found, -1 not a valid IP address."""
        bs = [_b(s) for s in symbols]
        off = np.zeros(len(bs) + 1, dtype=np.uint64)
        if bs:
            off[1:] = np.cumsum([len(b) for b in bs])
        blob = np.frombuffer(b"".join(bs) + b"\0", dtype=np.uint8)
        out = np.zeros(len(bs), dtype=np.int8)
        nets = ctypes.create_string_buffer(self.nets, max(len(self.nets), 1))
        self.lib.oracle_iplist_check(nets, ctypes.c_size_t(self.n), blob.ctypes.data_as(ctypes.c_void_p),
                                     off.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(len(bs)),
                                     out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(threads))
        return out


class RegexList:
    """parseRegexList (regexList.go:44-65): non-empty lines then overrides, each regexp.Compile'd
    (the first error fails the list); checkList: any pattern matches (Go regexp restatement in C,
    oracle/goregex.c, OpenMP over symbols)."""

    def __init__(self, lines, overrides=()):
        self.pats = [_b(p) for p in [x for x in lines if _b(x)] + list(overrides)]
        if self.pats:  # compile errors surface here, as parseRegexList returns them
            self._found([b""])

    def num_entries(self):
        return len(self.pats)

    def _found(self, symbols, threads=1):
        import oracle
        L = oracle.lib()
        pb, po = _blob(self.pats)
        sb, so = _blob([_b(s) for s in symbols])
        out = np.zeros(len(symbols), dtype=np.int8)
        err = ctypes.create_string_buffer(600)
        rc = L.oracle_regex_list_found(pb.ctypes.data, po.ctypes.data, len(self.pats), sb.ctypes.data, so.ctypes.data,
                                       len(symbols), out.ctypes.data, threads, err, len(err))
        if rc:
            raise ListParseError(err.value.decode("utf-8", "surrogateescape"))
        return out

    def found(self, symbols, threads=16):
        return self._found(symbols, threads)


def _blob(items):
    off = np.zeros(len(items) + 1, dtype=np.uint64)
    if items:
        off[1:] = np.cumsum([len(x) for x in items])
    return np.frombuffer(b"".join(items) + b"\0", dtype=np.uint8), off


def codes(found: np.ndarray, blacklist: bool) -> np.ndarray:
    """HandleListEntry's status code per symbol from found (1 / 0 / -1 = check error)."""
    if blacklist:
        c = np.where(found == 1, PERMISSION_DENIED, OK)
    else:
        c = np.where(found == 1, OK, NOT_FOUND)
    return np.where(found < 0, INVALID_ARGUMENT, c).astype(np.int32)
