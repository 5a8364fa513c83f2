"""ORACLE (test infrastructure only) -- Python glue over the CPU restatement.

    compile (oracle/goexpr.py + oracle/ilcompile.py, Python)  ->  IL program words + string table
    interpret (oracle/il_interp.c, C, liboracle.so)           ->  Go-faithful results per (bag, rule)

`OracleEvaluator` mirrors `expr.Evaluator` as implemented by `evaluator.IL`
(mixer/pkg/il/evaluator/evaluator.go:36-200): Eval / EvalPredicate on an expression text and a bag.
`oracle_matrix` gives the per-pair {false, true, error, panic} codes that the GPU engine's parity
tests compare against.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use it.
"""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import goexpr  # noqa: E402
import ilcompile  # noqa: E402
from govalue import GoDuration, GoFloat64, GoInt64, GoTime, bytes_go_str, go_str_bytes  # noqa: E402

_LIB = None


def build(force=False):
    """Compile liboracle.so with the committed Makefile (gcc)."""
    so = os.path.join(_HERE, "liboracle.so")
    srcs = [os.path.join(_HERE, f) for f in os.listdir(_HERE) if f.endswith((".c", ".h"))]
    if force or not os.path.exists(so) or any(os.path.getmtime(s) > os.path.getmtime(so) for s in srcs):
        subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])
    return so


class _Gv(ctypes.Structure):
    _fields_ = [("k", ctypes.c_uint8), ("inl_used", ctypes.c_uint8), ("len", ctypes.c_uint32),
                ("p", ctypes.c_void_p), ("i", ctypes.c_int64), ("ns", ctypes.c_int32),
                ("inl", ctypes.c_uint8 * 16)]


class _Result(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("rtype", ctypes.c_int32), ("v1", ctypes.c_uint32),
                ("v2", ctypes.c_uint32), ("val", _Gv), ("msg", ctypes.c_char * 512)]


# `matches`: the C interpreter runs the C restatement of Go's regexp (goregex.c); goregex.py is the
# Python form of the same restatement, kept for the known-answer tests (the two are compared there)


def lib():
    global _LIB
    if _LIB is None:
        so = build()
        L = ctypes.CDLL(so)
        L.oracle_prog_new.restype = ctypes.c_void_p
        L.oracle_prog_new.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
        L.oracle_prog_free.argtypes = [ctypes.c_void_p]
        L.oracle_eval.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                  ctypes.POINTER(_Result)]
        L.oracle_eval_matrix.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                         ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]
        L.oracle_result_size.restype = ctypes.c_size_t
        assert L.oracle_result_size() == ctypes.sizeof(_Result), "oracle_result layout mismatch"
        L.oracle_referenced.restype = ctypes.c_int64
        L.oracle_referenced.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                        ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
        L.oracle_regex_match.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_regex_cache.argtypes = [ctypes.c_int]
        L.oracle_regex_list_found.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int,
                                              ctypes.c_void_p, ctypes.c_size_t]
        # string lists (lists_oracle.c): Go map + strings.ToUpper, the table of oracle/unicode_upper.json
        L.oracle_upper_table.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_go_to_upper.restype = ctypes.c_size_t
        L.oracle_go_to_upper.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.oracle_strlist_new.restype = ctypes.c_void_p
        L.oracle_strlist_new.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        L.oracle_strlist_entries.restype = ctypes.c_size_t
        L.oracle_strlist_entries.argtypes = [ctypes.c_void_p]
        L.oracle_strlist_free.argtypes = [ctypes.c_void_p]
        L.oracle_strlist_found.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.c_void_p, ctypes.c_int]
        import json
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "unicode_upper.json")) as f:
            pairs = sorted(json.load(f)["pairs"])
        import numpy as _np
        _UPPER_PAIRS = _np.array(pairs, dtype=_np.uint32).reshape(-1)
        L.oracle_upper_table(_UPPER_PAIRS.ctypes.data, len(pairs))
        # memquota C restatement (memquota_oracle.c)
        L.mq_create.restype = ctypes.c_void_p
        L.mq_create.argtypes = [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
        L.mq_destroy.argtypes = [ctypes.c_void_p]
        L.mq_handle_batch.restype = ctypes.c_int
        L.mq_handle_batch.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int]
        _LIB = L
    return _LIB


def regex_match(pattern, subject):
    """regexp.MatchString(pattern, subject) by the C restatement -> (1 | 0 | -1 | -2, error text)."""
    L = lib()
    p = pattern.encode("utf-8", "surrogateescape") if isinstance(pattern, str) else bytes(pattern)
    q = subject.encode("utf-8", "surrogateescape") if isinstance(subject, str) else bytes(subject)
    err = ctypes.create_string_buffer(600)
    m = L.oracle_regex_match(p, len(p), q, len(q), err, len(err))
    return m, err.value.decode("utf-8", "surrogateescape") if m < 0 else ""


def regex_cache(on: bool):
    """The C `matches` compiles each pattern once per thread (on, default) or on every call, as
    regexp.MatchString does (off: the CPU baseline's faithful cost)."""
    lib().oracle_regex_cache(1 if on else 0)


# mixer/pkg/il/runtime/externs.go:30-39 -- (params, return) il types of the standard externs
EXTERN_SIGS = {
    "ip": ([ilcompile.T_STRING], ilcompile.T_INTERFACE),
    "ip_equal": ([ilcompile.T_INTERFACE, ilcompile.T_INTERFACE], ilcompile.T_BOOL),
    "timestamp": ([ilcompile.T_STRING], ilcompile.T_INTERFACE),
    "timestamp_equal": ([ilcompile.T_INTERFACE, ilcompile.T_INTERFACE], ilcompile.T_BOOL),
    "match": ([ilcompile.T_STRING, ilcompile.T_STRING], ilcompile.T_BOOL),
    "matches": ([ilcompile.T_STRING, ilcompile.T_STRING], ilcompile.T_BOOL),
    "startsWith": ([ilcompile.T_STRING, ilcompile.T_STRING], ilcompile.T_BOOL),
    "endsWith": ([ilcompile.T_STRING, ilcompile.T_STRING], ilcompile.T_BOOL),
}


class OracleProgram:
    """An IL program loaded into the C interpreter (interpreter.New adds the extern defs,
    interpreter.go:80-93)."""

    def __init__(self, program: ilcompile.Program):
        for name, (params, ret) in EXTERN_SIGS.items():
            program.add_extern_def(name, params, ret)
        self.program = program
        st = program.strings
        nstr = len(st.strs)
        enc = [go_str_bytes(s) for s in st.strs]
        offs = np.zeros(nstr + 1, dtype=np.uint64)
        offs[1:] = np.cumsum([len(b) for b in enc])
        blob = np.frombuffer(b"".join(enc) + b"\0", dtype=np.uint8).copy()
        kind = np.zeros(nstr, dtype=np.uint8)
        addr = np.zeros(nstr, dtype=np.uint32)
        ret = np.zeros(nstr, dtype=np.uint8)
        poff = np.zeros(nstr, dtype=np.uint32)
        npar = np.zeros(nstr, dtype=np.uint8)
        params = []
        for fid, f in program.functions.items():
            kind[fid] = 2 if f.address == 0 else 1
            addr[fid] = f.address
            ret[fid] = f.ret
            poff[fid] = len(params)
            npar[fid] = len(f.params)
            params.extend(f.params)
        par = np.array(params + [0], dtype=np.uint8)
        code = np.array(program.code, dtype=np.uint32)
        self._keep = (code, blob, offs, kind, addr, ret, poff, npar, par)
        L = lib()
        self.h = L.oracle_prog_new(code.ctypes.data, len(code), blob.ctypes.data, offs.ctypes.data, nstr,
                                   kind.ctypes.data, addr.ctypes.data, ret.ctypes.data, poff.ctypes.data,
                                   npar.ctypes.data, par.ctypes.data, len(params))

    def fn_id(self, name="eval"):
        return self.program.strings.try_get_id(name)

    def __del__(self):
        if getattr(self, "h", None) and _LIB is not None:
            _LIB.oracle_prog_free(self.h)
            self.h = None

    def run(self, batch, req: int, fn="eval"):
        """Interpreter.Eval(fn, bag) -> ('ok', value) | ('error', msg) | ('panic', msg)."""
        r = _Result()
        lib().oracle_eval(self.h, self.fn_id(fn), ctypes.byref(batch.c_struct()), req, ctypes.byref(r))
        msg = r.msg.decode("utf-8", "surrogateescape")
        if r.status == 1:
            return "error", msg
        if r.status == 2:
            return "panic", msg
        return "ok", _result_value(r, batch)


def eval_il(program: ilcompile.Program, fn: str, batch, req: int = 0):
    """interpreter.New(program, nil).Eval(fn, bag) (interpreter.go:62-69): ('ok', value) |
    ('error', msg) | ('panic', msg)."""
    if program.get(fn) is None:
        return "error", "function not found: '%s'" % fn
    return OracleProgram(program).run(batch, req, fn)


def _result_value(r: _Result, batch):
    """interpreter.Result.AsInterface (result.go:99-116)."""
    t = r.rtype
    if t == ilcompile.T_BOOL:
        return r.v1 != 0
    if t == ilcompile.T_INTEGER:
        return GoInt64(ilcompile.words_to_int(r.v1, r.v2))
    if t == ilcompile.T_DURATION:
        return GoDuration(ilcompile.words_to_int(r.v1, r.v2))
    if t == ilcompile.T_DOUBLE:
        return GoFloat64(ilcompile.words_to_double(r.v1, r.v2))
    if t == ilcompile.T_VOID:
        return None
    v = r.val
    if t == ilcompile.T_STRING:
        return bytes_go_str(ctypes.string_at(v.p, v.len)) if v.len else ""
    if t == ilcompile.T_INTERFACE:
        k = v.k
        if k == 1:
            return bytes_go_str(ctypes.string_at(v.p, v.len)) if v.len else ""
        if k == 7:
            return bytes(v.inl) if v.inl_used else (ctypes.string_at(v.p, v.len) if v.len else b"")
        if k == 6:
            return GoTime(v.i, v.ns)
        if k == 2:
            return GoInt64(v.i)
        if k == 4:
            return bool(v.i)
        if k == 5:
            return GoDuration(v.i)
        if k == 3:
            return GoFloat64(struct.unpack("<d", struct.pack("<q", v.i))[0])
        if k == 8:
            a, b = int(batch.map_offsets[v.i]), int(batch.map_offsets[v.i + 1])
            return {bytes_go_str(batch.string(int(batch.map_keys[e]))): bytes_go_str(batch.string(int(batch.map_values[e])))
                    for e in range(a, b)}
        return None
    return None


class OracleEvaluator:
    """evaluator.IL restated (evaluator.go:36-200) with an unbounded expression cache."""

    def __init__(self, manifest: dict, fmap=None):
        self.attrs = {k: (goexpr.VT[v] if isinstance(v, str) else v) for k, v in manifest.items()}
        self.fmap = fmap if fmap is not None else goexpr.func_map()
        self.cache = {}

    def compile(self, text):
        """-> OracleProgram, or raises with the reference's error text."""
        p = self.cache.get(text)
        if p is None:
            prog, _ = ilcompile.compile_expr(text, self.attrs, self.fmap)
            p = OracleProgram(prog)
            self.cache[text] = p
        return p

    def eval(self, text, batch, req: int):
        try:
            p = self.compile(text)
        except (goexpr.ParseError, goexpr.TypeCheckError, ilcompile.CompileError) as e:
            return "error", str(e)
        except goexpr.EvalPanic as e:
            return "panic", str(e)
        return p.run(batch, req)

    def eval_predicate(self, text, batch, req: int):
        st, v = self.eval(text, batch, req)
        if st == "ok" and not isinstance(v, bool):
            return "panic", "interpreter.Result: result is not bool"
        return st, v


# per-pair codes
FALSE, TRUE, ERROR, PANIC = 0, 1, 2, 3


def oracle_matrix(evaluator: OracleEvaluator, rules, batch, req_begin=0, req_end=None, threads=8):
    """codes[r, k] for EvalPredicate(rules[k], bag r) over requests [req_begin, req_end)."""
    if req_end is None:
        req_end = batch.n
    nreq = req_end - req_begin
    codes = np.zeros((nreq, len(rules)), dtype=np.uint8)
    progs = []
    static = {}
    for k, text in enumerate(rules):
        try:
            progs.append(evaluator.compile(text))
        except (goexpr.ParseError, goexpr.TypeCheckError, ilcompile.CompileError):
            static[k] = ERROR
            progs.append(None)
        except goexpr.EvalPanic:
            static[k] = PANIC
            progs.append(None)
    live = [k for k in range(len(rules)) if progs[k] is not None]
    if live:
        handles = (ctypes.c_void_p * len(live))(*[progs[k].h for k in live])
        fids = np.array([progs[k].fn_id() for k in live], dtype=np.uint32)
        sub = np.zeros((nreq, len(live)), dtype=np.uint8)
        lib().oracle_eval_matrix(handles, fids.ctypes.data, len(live), ctypes.byref(batch.c_struct()),
                                 req_begin, req_end, sub.ctypes.data, threads)
        codes[:, live] = sub
    for k, c in static.items():
        codes[:, k] = c
    return codes


def oracle_referenced(evaluator: OracleEvaluator, rules, batch, req: int):
    """FakeBag.ReferencedList (il/testing/fakebag.go:75-89) of request `req` after EvalPredicate of
    every rule in order: sorted distinct "name" / "name[key]" strings (bytes).  Rules that fail to
    compile read nothing (evaluator.go:157-179 returns the compile error before touching the bag)."""
    progs = []
    for text in rules:
        try:
            progs.append(evaluator.compile(text))
        except (goexpr.ParseError, goexpr.TypeCheckError, ilcompile.CompileError, goexpr.EvalPanic):
            pass
    if not progs:
        return []
    handles = (ctypes.c_void_p * len(progs))(*[p.h for p in progs])
    fids = np.array([p.fn_id() for p in progs], dtype=np.uint32)
    cap = 4096
    while True:
        buf = ctypes.create_string_buffer(cap)
        n = lib().oracle_referenced(handles, fids.ctypes.data, len(progs), ctypes.byref(batch.c_struct()), req,
                                    buf, cap)
        if n >= 0:
            return [x for x in buf.raw[:n].split(b"\n") if x]
        cap = -n + 16
