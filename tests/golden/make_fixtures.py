#!/usr/bin/env python3
"""Extract the reference's Go test tables into JSON fixtures (data only).

Run in the build container, where the read-only reference is mounted:

    python tests/golden/make_fixtures.py [/root/reference]

Outputs (committed):
  tests/golden/ilt_tests.json      <- mixer/pkg/il/testing/tests.go:37-2258 (TestData) and the two
                                      attribute manifests at tests.go:2342-2489
  tests/golden/expr_parse.json     <- mixer/pkg/expr/expr_test.go:27-76 (TestGoodParse postfix forms)
  tests/golden/manifest_testdata.json <- mixer/testdata/config/attributes.yaml (names + ValueType)
  tests/golden/il_interpreter.json <- mixer/pkg/il/interpreter/interpreter_test.go (every IL-level case)
  tests/golden/il_read.json        <- mixer/pkg/il/text/read_test.go:28-427 (assembler round trips, errors)
  tests/golden/expr_checks.json    <- mixer/pkg/expr/expr_test.go:190-333 (bad parses, type checks)
  tests/golden/externs_kat.json    <- mixer/pkg/il/runtime/externs_test.go:24-129 (extern KATs)
  tests/golden/list_cases.json     <- mixer/adapter/list/list_test.go (list configurations and cases)
  tests/golden/resolver_cases.json <- mixer/pkg/runtime/resolver_test.go:38-145 (TestResolver_Resolve)
  tests/golden/memquota_cases.json <- mixer/adapter/memquota/{memquota,rollingWindow}_test.go
  tests/golden/protobag_cases.json <- mixer/pkg/attribute/bag_test.go (CompressedAttributes + Get results)

Values are tagged by their Go dynamic type so the Go semantics that matter (int64 vs int, []byte vs
string, time.Duration vs int64) survive the trip through JSON.
"""
from __future__ import annotations

import calendar
import datetime
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gosrc  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def _ts(y, mo, d, h, mi, s):
    return calendar.timegm(datetime.datetime(y, mo, d, h, mi, s).timetuple())


# Named values declared at mixer/pkg/il/testing/tests.go:29-34.
NAMED = {
    "duration19": {"t": "duration", "v": str(19_000_000)},
    "duration20": {"t": "duration", "v": str(20_000_000)},
    "time1999": {"t": "time", "sec": str(_ts(1999, 12, 31, 23, 59, 0)), "nsec": 0},
    "time1977": {"t": "time", "sec": str(_ts(1977, 2, 4, 12, 0, 0)), "nsec": 0},
    "t": {"t": "time", "sec": str(_ts(2015, 1, 2, 15, 4, 35)), "nsec": 0},
    "t2": {"t": "time", "sec": str(_ts(2015, 1, 2, 15, 4, 34)), "nsec": 0},
    "time.RFC3339": {"t": "string", "v": "2006-01-02T15:04:05Z07:00"},
    "net.IPv4zero": {"t": "bytes", "v": "00000000000000000000ffff00000000"},
    # interpreter_test.go:87 (duration20ms, _ := time.ParseDuration("20ms")) and time constants
    "duration20ms": {"t": "duration", "v": str(20_000_000)},
    "time.Hour": {"t": "duration", "v": str(3600 * 10**9)},
    "time.Minute": {"t": "duration", "v": str(60 * 10**9)},
    "time.Second": {"t": "duration", "v": str(10**9)},
    "time.Millisecond": {"t": "duration", "v": str(10**6)},
    "nil": {"t": "nil"},
}


def _arith(op, a, b):
    """Go constant arithmetic on two converted values (+ / -): strings concatenate, durations and
    integers add exactly, float64 values round once per operation like IEEE doubles."""
    if op == "+" and a["t"] == b["t"] == "string":
        return {"t": "string", "v": a["v"] + b["v"]}
    assert a["t"] == b["t"] and a["t"] in ("duration", "int64", "int", "float64"), (a, b)
    if a["t"] == "float64":
        x, y = float(a["v"]), float(b["v"])
        return {"t": "float64", "v": repr(x + y if op == "+" else x - y)}
    x, y = int(a["v"]), int(b["v"])
    return {"t": a["t"], "v": str(x + y if op == "+" else x - y)}


def parse_ipv4_16(s):
    parts = [int(p) for p in s.split(".")]
    return "00000000000000000000ffff" + "".join("%02x" % p for p in parts)


def go_int(text):
    return int(text, 16) if text.lower().startswith("0x") else int(text, 10)


def conv(node):
    """Convert a parsed Go value node into a tagged JSON value."""
    kind = node[0]
    if kind == "str":
        return {"t": "string", "v": node[1]}
    if kind == "num":
        if re.match(r"^(0[xX][0-9a-fA-F]+|\d+)$", node[1]):
            return {"t": "int", "v": str(go_int(node[1]))}
        return {"t": "float_untyped", "v": node[1]}
    if kind == "ident":
        name = node[1]
        if name in ("true", "false"):
            return {"t": "bool", "v": name == "true"}
        if name in NAMED:
            return NAMED[name]
        if name.startswith("descriptor.") or name.startswith("dpb."):
            return {"t": "valuetype", "v": name.split(".", 1)[1]}
        return {"t": "ident", "v": name}
    if kind in ("concat", "sub"):
        return _arith("+" if kind == "concat" else "-", conv(node[1]), conv(node[2]))
    if kind == "mul":  # duration * integer constant
        a, b = conv(node[1]), conv(node[2])
        if a["t"] != "duration":
            a, b = b, a
        assert a["t"] == "duration" and b["t"] == "int", (a, b)
        return {"t": "duration", "v": str(int(a["v"]) * int(b["v"]))}
    if kind == "call":
        name, args = node[1], node[2]
        if name == "int64":
            a = conv(args[0])
            return {"t": "int64", "v": a["v"]}
        if name == "float64":
            return {"t": "float64", "v": repr(float(conv(args[0])["v"]))}
        if name == "net.ParseIP":
            return {"t": "bytes", "v": parse_ipv4_16(conv(args[0])["v"])}
        if name == "time.Date":  # time.Date(y, mo, d, h, mi, s, ns, time.UTC)
            y, mo, d, h, mi, sec, ns = [int(conv(x)["v"]) for x in args[:7]]
            return {"t": "time", "sec": str(_ts(y, mo, d, h, mi, sec)), "nsec": ns}
        if name == "time.Unix":
            return {"t": "time", "sec": conv(args[0])["v"], "nsec": int(conv(args[1])["v"])}
        if name == "ExternFromFn":  # a test-defined Go function: only its name travels
            return {"t": "extern", "v": conv(args[0])["v"]}
        raise ValueError("unknown call %s" % name)
    if kind == "conv":
        typ, arg = node[1], node[2]
        inner = conv(arg)
        if typ in ("[]uint8", "[]byte"):
            assert inner["t"] == "bytes", inner
            return inner
        raise ValueError("unknown conversion %s" % typ)
    if kind == "composite":
        typ, elems = node[1], node[2]
        if typ == "[]byte" or typ == "[]uint8":
            return {"t": "bytes", "v": "".join("%02x" % go_int(e[1][1]) for e in elems)}
        if typ == "map[string]string":
            return {"t": "map", "v": {conv(k)["v"]: conv(v)["v"] for k, v in elems}}
        if typ == "map[string]interface{}":
            return {"t": "bag", "v": {conv(k)["v"]: conv(v) for k, v in elems}}
        if typ == "[]string":
            return {"t": "strings", "v": [conv(v)["v"] for _, v in elems]}
        if typ == "map[string]Extern":
            return {"t": "externs", "v": sorted(conv(k)["v"] for k, _ in elems)}
        return {"t": "composite", "typ": typ, "v": [[None if k is None else conv(k), conv(v)] for k, v in elems]}
    if kind == "func":
        return {"t": "func", "v": node[1]}
    if kind == "neg":
        a = conv(node[1])
        v = a["v"][1:] if a["v"].startswith("-") else "-" + a["v"]
        return {"t": a["t"], "v": v}
    raise ValueError(node)


def fn_metadata(node):
    out = []
    for _, fm in node[2]:
        d = {"Name": "", "Instance": False, "TargetType": "VALUE_TYPE_UNSPECIFIED",
             "ReturnType": "VALUE_TYPE_UNSPECIFIED", "ArgumentTypes": []}
        for k, v in fm[2]:
            key = k[1]
            if key == "Name":
                d["Name"] = v[1]
            elif key == "Instance":
                d["Instance"] = v[1] == "true"
            elif key in ("TargetType", "ReturnType"):
                d[key] = v[1].split(".", 1)[1]
            elif key == "ArgumentTypes":
                d[key] = [e[1][1].split(".", 1)[1] for e in v[2]]
        out.append(d)
    return out


def extract_ilt(ref):
    path = os.path.join(ref, "mixer/pkg/il/testing/tests.go")
    src = open(path, encoding="utf-8").read()
    table = gosrc.find_var(src, "TestData")
    rows = []
    for idx, (_, entry) in enumerate(table[2]):
        assert entry[0] == "composite"
        row = {"index": idx}
        for k, v in entry[2]:
            key = k[1]
            if key == "Fns":
                row["Fns"] = fn_metadata(v)
            elif key == "Externs":
                row["Externs"] = sorted(conv(kk)["v"] for kk, _ in v[2])
            elif key == "conf":
                row["conf"] = v[1]
            elif key == "I":
                row["I"] = conv(v)["v"]
            else:
                cv = conv(v)
                row[key] = cv if key == "R" else cv["v"]
        rows.append(row)
    manifests = {}
    for name in ("exprEvalAttrs", "defaultAttrs"):
        m = gosrc.find_var(src, name)
        attrs = {}
        for k, v in m[2]:
            (_, vt), = [(kk, vv) for kk, vv in v[2]]
            attrs[conv(k)["v"]] = vt[1].split(".", 1)[1]
        manifests[name] = attrs
    return {"source": "mixer/pkg/il/testing/tests.go", "rows": rows, "manifests": manifests}


def extract_parse(ref):
    path = os.path.join(ref, "mixer/pkg/expr/expr_test.go")
    src = open(path, encoding="utf-8").read()
    m = re.search(r"func TestGoodParse\(t \*testing.T\) \{\s*tests := \[\]struct \{(?:[^{}]|\{\})*\}\{", src)
    p = gosrc.Parser(src, m.end() - 1)
    lit = p.parse_composite("[]struct")
    cases = [[conv(e[1][2][0][1])["v"], conv(e[1][2][1][1])["v"]] for e in lit[2]]
    return {"source": "mixer/pkg/expr/expr_test.go:27-76", "cases": cases}


def _func_body(src, name):
    """Text of `func <name>(t *testing.T) { ... }`."""
    m = re.search(r"^func %s\(t \*testing\.T\) \{" % re.escape(name), src, re.M)
    p = gosrc.Parser(src, m.end() - 1)
    return p.skip_balanced("{", "}"), m.end() - 1


def _test_map(src, start):
    """The `var tests = map[string]test{...}` literal after `start` -> {name: {field: value}}."""
    m = re.compile(r"var tests = map\[string\]test\{").search(src, start)
    p = gosrc.Parser(src, m.end() - 1)
    lit = p.parse_composite("map[string]test")
    out = {}
    for k, v in lit[2]:
        fields = {}
        for fk, fv in v[2]:
            cv = conv(fv)
            fields[fk[1]] = cv if fk[1] in ("expected", "input") else cv["v"]
        out[conv(k)["v"]] = fields
    return out


def _raw_after(src, start, marker):
    """The raw string literal that follows `marker` after `start`."""
    i = src.index(marker, start)
    j = src.index("`", i)
    return src[j + 1:src.index("`", j + 1)]


def _case(name, fields, fn="main"):
    c = {"name": name, "code": fields.get("code", ""), "fn": fn}
    if "input" in fields:
        c["input"] = fields["input"]["v"]
    if fields.get("err"):
        c["err"] = fields["err"]
    else:
        c["expected"] = fields.get("expected", {"t": "nil"})
    if "externs" in fields:
        c["externs"] = fields["externs"]
    return c


def extract_interpreter(ref):
    """mixer/pkg/il/interpreter/interpreter_test.go: every IL-level case (TestInterpreter_Eval and its
    parent-code inheritance, the stack-underflow / stack-overflow / heap-overflow templates, the
    underflowing `ret` per type, EvalFnID and the unknown-function error), as the final IL text plus
    the input bag, the expected value or error, and the names of test-defined Go externs."""
    path = os.path.join(ref, "mixer/pkg/il/interpreter/interpreter_test.go")
    src = open(path, encoding="utf-8").read()
    cases = []
    # TestInterpreter_EvalFnID / TestInterpreter_Eval_FunctionNotFound (:48-83)
    for tname, fn, exp in (("TestInterpreter_EvalFnID", "main", {"expected": {"t": "bool", "v": False}}),
                           ("TestInterpreter_Eval_FunctionNotFound", "foo", None)):
        body, at = _func_body(src, tname)
        code = _raw_after(src, at, "text.ReadText(")
        if exp is None:
            err = re.search(r'e\.Error\(\) != "([^"]*)"', body).group(1)
            cases.append({"name": tname, "code": code, "fn": fn, "err": err})
        else:
            cases.append({"name": tname, "code": code, "fn": fn, **exp})
    # TestInterpreter_Eval: a case without code runs its parent's ("a/b" -> "a")
    _, at = _func_body(src, "TestInterpreter_Eval")
    tests = _test_map(src, at)
    for n in sorted(tests):
        f = dict(tests[n])
        if not f.get("code"):
            f["code"] = tests[n[:n.rindex("/")]]["code"]
        cases.append(_case("Eval/" + n, f))
    # the templated tables: code spliced into the function's template, one error for all
    for tname in ("TestInterpreter_Eval_StackUnderflow", "TestInterpreter_Eval_StackOverflow",
                  "TestInterpreter_Eval_HeapOverflow"):
        body, at = _func_body(src, tname)
        tests = _test_map(src, at)
        tmpl = _raw_after(src, at, "template := ")
        err = re.search(r'test\.err = "([^"]*)"', body).group(1)
        inp = None
        m = re.search(r"test\.input = ", body)
        if m:
            p = gosrc.Parser(src, at + m.end())
            inp = conv(p.parse_value())
        for n in sorted(tests):
            f = dict(tests[n])
            f["code"] = tmpl.replace("%s", f["code"], 1)
            f["err"] = err
            if inp is not None:
                f["input"] = inp
            cases.append(_case(tname[len("TestInterpreter_"):] + "/" + n, f))
    # TestInterpreter_Eval_StackUnderflow_Ret: `ret` on an empty stack, per return type
    body, at = _func_body(src, "TestInterpreter_Eval_StackUnderflow_Ret")
    types = gosrc.Parser(src, src.index("var types = ", at) + len("var types = ")).parse_value()
    tmpl = _raw_after(src, at, "fmt.Sprintf(")
    err = re.search(r'err:\s*"([^"]*)"', body).group(1)
    for _, ty in types[2]:
        cases.append({"name": "StackUnderflow_Ret_" + ty[1], "code": tmpl.replace("%s", ty[1], 1), "fn": "main",
                      "err": err})
    return {"source": "mixer/pkg/il/interpreter/interpreter_test.go", "cases": cases}


def extract_read(ref):
    """mixer/pkg/il/text/read_test.go:28-427 (readTests): IL text in, WriteText form or error out."""
    src = open(os.path.join(ref, "mixer/pkg/il/text/read_test.go"), encoding="utf-8").read()
    rows = []
    for _, e in gosrc.find_var(src, "readTests")[2]:
        rows.append({k[1]: conv(v)["v"] for k, v in e[2]})
    return {"source": "mixer/pkg/il/text/read_test.go:28-427", "cases": rows}


def _struct_table(src, func):
    """The `tests := []struct{...}{...}` (or `var cases = ...`) literal of `func` -> element nodes."""
    m = re.search(r"func %s\(t \*testing.T\) \{.*?(?:tests :=|var cases =) \[\]struct \{(?:[^{}]|\{\})*\}\{" % func, src,
                  re.S)
    return gosrc.Parser(src, m.end() - 1).parse_composite("[]struct")[2]


def extract_expr_checks(ref):
    """mixer/pkg/expr/expr_test.go: TestBadParse (:190-246, source -> error fragment) and
    TestInternalTypeCheck (:258-333, expression + attributes + extra functions -> return type or
    error fragment; "__SUCCESS__" = type-checks)."""
    src = open(os.path.join(ref, "mixer/pkg/expr/expr_test.go"), encoding="utf-8").read()
    bad = [[conv(e[1][2][0][1])["v"], conv(e[1][2][1][1])["v"]] for e in _struct_table(src, "TestBadParse")]
    checks = []
    for _, e in _struct_table(src, "TestInternalTypeCheck"):
        f = [v for _, v in e[2]]
        attrs = {}
        for _, ad in f[2][2]:
            if ad[2]:
                attrs[conv(ad[2][0][1])["v"]] = conv(ad[2][1][1])["v"]
        fns = []
        if f[3][0] == "composite":
            for _, fm in f[3][2]:
                d = {"Name": "", "Instance": False, "TargetType": "VALUE_TYPE_UNSPECIFIED",
                     "ReturnType": "VALUE_TYPE_UNSPECIFIED", "ArgumentTypes": []}
                for k, v in fm[2]:
                    if k[1] == "Name":
                        d["Name"] = conv(v)["v"]
                    elif k[1] == "Instance":
                        d["Instance"] = conv(v)["v"]
                    elif k[1] in ("TargetType", "ReturnType"):
                        d[k[1]] = conv(v)["v"]
                    elif k[1] == "ArgumentTypes":
                        d["ArgumentTypes"] = [conv(x)["v"] for _, x in v[2]]
                fns.append(d)
        err = "__SUCCESS__" if f[4] == ("ident", "success") else conv(f[4])["v"]
        checks.append({"s": conv(f[0])["v"], "ret": conv(f[1])["v"], "attrs": attrs, "fns": fns, "err": err})
    return {"source": "mixer/pkg/expr/expr_test.go:190-333", "bad_parse": bad, "type_checks": checks}


def extract_externs(ref):
    """mixer/pkg/il/runtime/externs_test.go:24-129: the extern KATs as (extern, arguments, expected)."""
    src = open(os.path.join(ref, "mixer/pkg/il/runtime/externs_test.go"), encoding="utf-8").read()
    cases = []
    body, _ = _func_body(src, "TestExternIp")
    a = re.search(r'externIP\("([^"]*)"\)', body).group(1)
    b = re.search(r'net\.ParseIP\("([^"]*)"\)', body).group(1)
    cases.append({"fn": "ip", "args": [a], "want": {"t": "bytes", "v": parse_ipv4_16(b)}})
    body, _ = _func_body(src, "TestExternIp_Error")
    cases.append({"fn": "ip", "args": [re.search(r'externIP\("([^"]*)"\)', body).group(1)], "err": True})
    for name, want in (("TestExternIpEqual_True", True), ("TestExternIpEqual_False", False)):
        body, _ = _func_body(src, name)
        cases.append({"fn": "ip_equal", "args": re.findall(r'net\.ParseIP\("([^"]*)"\)', body), "want": want})
    body, _ = _func_body(src, "TestExternTimestamp")
    ts = re.search(r'externTimestamp\("([^"]*)"\)', body).group(1)
    m = re.search(r"ti\.Year\(\) != (\d+) \|\| ti\.Month\(\) != time\.(\w+) \|\| ti\.Day\(\) != (\d+) \|\| "
                  r"ti\.Hour\(\) != (\d+) \|\| ti\.Minute\(\) != (\d+)", body)
    month = ["January", "February", "March", "April", "May", "June", "July", "August", "September", "October",
             "November", "December"].index(m.group(2)) + 1
    cases.append({"fn": "timestamp", "args": [ts], "want_fields": [int(m.group(1)), month, int(m.group(3)),
                                                                  int(m.group(4)), int(m.group(5))]})
    body, _ = _func_body(src, "TestExternTimestamp_Error")
    cases.append({"fn": "timestamp", "args": [re.search(r'externTimestamp\("([^"]*)"\)', body).group(1)],
                  "err": True})
    for name, want in (("TestExternTimestampEqual_True", True), ("TestExternTimestampEqual_False", False)):
        body, _ = _func_body(src, name)
        cases.append({"fn": "timestamp_equal", "args": re.findall(r'externTimestamp\("([^"]*)"\)', body),
                      "want": want})
    for e in _struct_table(src, "TestExternMatch"):
        s_, p_, w = [conv(v) for _, v in e[1][2]]
        cases.append({"fn": "match", "args": [s_["v"], p_["v"]], "want": w["v"]})
    for e in _struct_table(src, "TestExternMatches"):
        p_, s_, w = [conv(v) for _, v in e[1][2]]
        cases.append({"fn": "matches", "args": [p_["v"], s_["v"]], "want": w["v"]})
    return {"source": "mixer/pkg/il/runtime/externs_test.go:24-129", "cases": cases}


LIST_TYPES = {"STRINGS": 0, "CASE_INSENSITIVE_STRINGS": 1, "IP_ADDRESSES": 2, "REGEX": 3}
RPC_CODES = {"OK": 0, "INVALID_ARGUMENT": 3, "NOT_FOUND": 5, "PERMISSION_DENIED": 7}


def _strings_after(body, marker):
    m = re.search(marker + r"\s*\[\]string\{", body)
    if not m:
        return None
    return [conv(v)["v"] for _, v in gosrc.Parser(body, m.end() - 1).parse_composite("[]string")[2]]


def extract_lists(ref):
    """mixer/adapter/list/list_test.go: each list test's configuration (entry type, overrides,
    blacklist), the served list and its (symbol, google.rpc code) cases.  TestIPList's second payload
    must fail to parse (the test checks only that); the expected text follows ipList.go:70's format
    with net.ParseCIDR's error for the entry."""
    src = open(os.path.join(ref, "mixer/adapter/list/list_test.go"), encoding="utf-8").read()
    ipfmt = re.search(r'fmt\.Errorf\("(could not parse list entry [^"]*)", orig, err\)',
                      open(os.path.join(ref, "mixer/adapter/list/ipList.go"), encoding="utf-8").read()).group(1)
    out = []
    for name in ("TestIPList", "TestStringList", "TestBlackStringList", "TestCaseInsensitiveStringList",
                 "TestNoUrlStringList", "TestRegexList"):
        body, _ = _func_body(src, name)
        spec = {"name": name, "type": LIST_TYPES[re.search(r"EntryType:\s*config\.(\w+)", body).group(1)],
                "overrides": _strings_after(body, r"Overrides:") or [],
                "blacklist": bool(re.search(r"Blacklist:\s*true", body))}
        m = re.search(r'listToServe := ("(?:[^"\\]|\\.)*")', body)
        if m:
            spec["entries"] = gosrc.go_unquote(m.group(1)).split("\n")
        else:
            spec["entries"] = _strings_after(body, r"WhiteList:") or []
        m = re.search(r"cases := \[\]struct \{(?:[^{}]|\{\})*\}\{", body)
        rows = gosrc.Parser(body, m.end() - 1).parse_composite("[]struct")[2]
        spec["cases"] = [[conv(e[1][2][0][1])["v"], RPC_CODES[e[1][2][1][1][1].split(".")[1]]] for e in rows]
        out.append(spec)
        if name == "TestIPList":  # "now try to parse a list with errors"
            i = body.index("now try to parse a list with errors")
            bad = _strings_after(body[i:], r"WhiteList:")
            entry = [e for e in bad if "." not in e][0]
            out.append({"name": name + " bad entry", "type": spec["type"], "entries": bad,
                        "overrides": spec["overrides"], "blacklist": False,
                        "parse_error": ipfmt.replace("%v", "%s") % (entry, "invalid CIDR address: %s/32" % entry)})
    return {"source": "mixer/adapter/list/list_test.go (TestIPList, TestStringList, TestBlackStringList, "
                      "TestCaseInsensitiveStringList, TestNoUrlStringList, TestRegexList). Codes: google.rpc OK 0, "
                      "INVALID_ARGUMENT 3, NOT_FOUND 5, PERMISSION_DENIED 7.", "lists": out}


# istio.io/api mixer/adapter/model/v1beta1 TemplateVariety (a dependency, not vendored in the reference)
TEMPLATE_VARIETY = {"TEMPLATE_VARIETY_CHECK": 0, "TEMPLATE_VARIETY_REPORT": 1, "TEMPLATE_VARIETY_QUOTA": 2,
                    "TEMPLATE_VARIETY_ATTRIBUTE_GENERATOR": 3}


def extract_resolver(ref):
    """mixer/pkg/runtime/resolver_test.go:38-145 (TestResolver_Resolve): rules are fakeRuleCfg
    {ns, ruleLength} entries, each one rule whose actions for the variety number ruleLength; the fake
    evaluator answers !selectReject, or selectError, for every rule."""
    rsrc = open(os.path.join(ref, "mixer/pkg/runtime/resolver.go"), encoding="utf-8").read()
    const = {k: re.search(r'\b%s = "([^"]*)"' % k, rsrc).group(1)
             for k in ("DefaultConfigNamespace", "DefaultIdentityAttribute", "ContextProtocolAttributeName")}
    src = open(os.path.join(ref, "mixer/pkg/runtime/resolver_test.go"), encoding="utf-8").read()
    saved = dict(NAMED)
    NAMED.update({"ia": {"t": "string", "v": const["DefaultIdentityAttribute"]},
                  "ns": {"t": "string", "v": const["DefaultConfigNamespace"]},
                  "ContextProtocolAttributeName": {"t": "string", "v": const["ContextProtocolAttributeName"]}})
    NAMED.update({"adptTmpl." + k: {"t": "int", "v": str(v)} for k, v in TEMPLATE_VARIETY.items()})
    try:
        m = re.search(r"tests := \[\]testcase\{", src)
        cases = []
        for _, e in gosrc.Parser(src, m.end() - 1).parse_composite("[]testcase")[2]:
            c = {"bag": {}, "rules": []}
            for k, v in e[2]:
                key = k[1]
                if key == "bag":
                    c["bag"] = {conv(kk)["v"]: conv(vv)["v"] for kk, vv in v[2]}
                elif key == "rules":
                    c["rules"] = [[conv(r[2][0][1])["v"], int(conv(r[2][1][1])["v"])] for _, r in v[2]]
                elif key in ("nactions", "callVariety", "variety"):
                    c[key] = int(conv(v)["v"])
                else:
                    c[key] = conv(v)["v"]
            c.setdefault("nactions", 0)
            cases.append(c)
    finally:
        NAMED.clear()
        NAMED.update(saved)
    return {"source": "mixer/pkg/runtime/resolver_test.go:38-145 (TestResolver_Resolve); rules are fakeRuleCfg "
                      "{ns, ruleLength} entries, each one rule whose actions for `variety` number ruleLength; the "
                      "fake evaluator returns !selectReject or selectError for every rule",
            "identity_attr": const["DefaultIdentityAttribute"], "default_ns": const["DefaultConfigNamespace"],
            "cases": cases}


def _struct_table_cols(src, func):
    """(column names, rows of converted values) of the `cases := []struct{...}{...}` table in `func`."""
    body, at = _func_body(src, func)
    m = re.search(r"cases := \[\]struct \{((?:[^{}]|\{\})*)\}\{", body)
    cols = re.findall(r"^\s*(\w+)\s+\S+\s*$", m.group(1), re.M)
    rows = gosrc.Parser(body, m.end() - 1).parse_composite("[]struct")[2]
    out = []
    for _, e in rows:
        vals = []
        for _, v in e[2]:
            c = conv(v)
            vals.append(c["v"] if c["t"] in ("string", "bool") else int(c["v"]))
        out.append(vals)
    return cols, out, body


def extract_memquota(ref):
    """mixer/adapter/memquota/memquota_test.go:64-197 (TestAllocAndRelease: quota limits, then per case
    an allocation and a release at a time offset) and rollingWindow_test.go (TestAlloc, TestRelease:
    newRollingWindow(limit, ticks) and its cases).  Durations in ns."""
    src = open(os.path.join(ref, "mixer/adapter/memquota/memquota_test.go"), encoding="utf-8").read()
    body, at = _func_body(src, "TestAllocAndRelease")
    m = re.search(r"limits := \[\]config\.Params_Quota\{", body)
    limits = {}
    for _, e in gosrc.Parser(body, m.end() - 1).parse_composite("[]config.Params_Quota")[2]:
        f = {k[1]: conv(v) for k, v in e[2]}
        limits[f["Name"]["v"]] = [int(f["MaxAmount"]["v"]), int(f["ValidDuration"]["v"])]
    cols, rows, _ = _struct_table_cols(src, "TestAllocAndRelease")
    cols = ["exp_ns" if c == "exp" else c for c in cols]
    out = {"alloc_and_release": {"limits": limits, "columns": cols, "cases": rows}}
    wsrc = open(os.path.join(ref, "mixer/adapter/memquota/rollingWindow_test.go"), encoding="utf-8").read()
    for func, key in (("TestAlloc", "window_alloc"), ("TestRelease", "window_release")):
        cols, rows, body = _struct_table_cols(wsrc, func)
        lim, ticks = re.search(r"newRollingWindow\((\d+), (\d+)\)", body).groups()
        out[key] = {"limit": int(lim), "ticks": int(ticks), "columns": cols, "cases": rows}
    out["source"] = ("mixer/adapter/memquota/memquota_test.go:64-197 (TestAllocAndRelease) and rollingWindow_test.go "
                     "(TestAlloc, TestRelease)")
    return out


def _int_map(node):
    return [[int(conv(k)["v"]), v] for k, v in node[2]]


def _compressed(node, local):
    """A mixerpb.CompressedAttributes literal -> the fixture's message dict (keys as in the test)."""
    out = {}
    for k, v in node[2]:
        f = k[1]
        if f == "Words":
            out["words"] = local[v[1]] if v[0] == "ident" else [conv(x)["v"] for _, x in v[2]]
            continue
        rows = _int_map(v)
        if f == "Strings":
            out["strings"] = [[a, int(conv(b)["v"])] for a, b in rows]
        elif f == "Int64S":
            out["int64s"] = [[a, int(conv(b)["v"])] for a, b in rows]
        elif f == "Doubles":
            out["doubles"] = [[a, float(conv(b)["v"])] for a, b in rows]
        elif f == "Bools":
            out["bools"] = [[a, conv(b)["v"]] for a, b in rows]
        elif f == "Timestamps":
            out["timestamps"] = [[a, [int(conv(b)["sec"]), conv(b)["nsec"]]] for a, b in rows]
        elif f == "Durations":
            out["durations"] = [[a, int(conv(b)["v"])] for a, b in rows]
        elif f == "Bytes":
            out["bytes"] = [[a, "".join("%02x" % go_int(e[1][1]) for e in b[2])] for a, b in rows]
        elif f == "StringMaps":
            out["string_maps"] = [[a, local[b[1]]] for a, b in rows]
    return out


def extract_protobag(ref):
    """mixer/pkg/attribute/bag_test.go: the CompressedAttributes messages of TestProtoBag, TestBogusProto,
    TestMessageDictEdge, TestDoubleStrings and TestReferenceTracking, their global word lists and the
    Get results each test asserts ({"t": "present"}: found, value not asserted; null: not found)."""
    path = os.path.join(ref, "mixer/pkg/attribute/bag_test.go")
    src = open(path, encoding="utf-8").read()
    saved = dict(NAMED)
    for name in ("t9", "d1"):  # package-level test values
        m = re.search(r"^\s*%s\s*=\s*" % name, src, re.M)
        NAMED[name] = conv(gosrc.Parser(src, m.end()).parse_value())
    cases = []
    try:
        for tname in ("TestProtoBag", "TestBogusProto", "TestMessageDictEdge", "TestDoubleStrings",
                      "TestReferenceTracking"):
            body, at = _func_body(src, tname)
            line0 = src[:at].count("\n") + 1
            local = {}
            for m in re.finditer(r"(\w+) := \[\]string\{", body):
                local[m.group(1)] = [conv(v)["v"] for _, v in
                                     gosrc.Parser(body, m.end() - 1).parse_composite("[]string")[2]]
            for m in re.finditer(r"(\w+) := mixerpb\.StringMap\{", body):
                sm = gosrc.Parser(body, m.end() - 1).parse_composite("mixerpb.StringMap")
                local[m.group(1)] = [[int(conv(k)["v"]), int(conv(v)["v"])] for k, v in sm[2][0][1][2]]
            m = re.search(r"attrs := mixerpb\.CompressedAttributes\{", body)
            msg = _compressed(gosrc.Parser(body, m.end() - 1).parse_composite("mixerpb.CompressedAttributes"), local)
            if tname == "TestProtoBag":
                m = re.search(r"cases := \[\]struct \{(?:[^{}]|\{\})*\}\{", body)
                rows = gosrc.Parser(body, m.end() - 1).parse_composite("[]struct")[2]
                get = []
                for _, e in rows:
                    name, val = conv(e[2][0][1])["v"], conv(e[2][1][1])
                    if val["t"] == "float_untyped":
                        val = {"t": "float64", "v": repr(float(val["v"]))}
                    elif val["t"] == "int":
                        val = {"t": "int64", "v": val["v"]}
                    elif val["t"] == "time":
                        val = {"t": "time", "sec": int(val["sec"]), "nsec": val["nsec"]}
                    get.append([name, val])
            elif tname == "TestBogusProto":
                m = re.search(r"cases := \[\]struct \{(?:[^{}]|\{\})*\}\{", body)
                get = [[conv(e[2][0][1])["v"], None] for _, e in gosrc.Parser(body, m.end() - 1).parse_composite("x")[2]]
            elif tname == "TestReferenceTracking":
                m = re.search(r"cases := \[\]struct \{(?:[^{}]|\{\})*\}\{", body)
                get = []
                for _, e in gosrc.Parser(body, m.end() - 1).parse_composite("x")[2]:
                    name, cond = conv(e[2][0][1])["v"], e[2][1][1]
                    if cond[0] == "ident":  # mixerpb.EXACT / ABSENCE; -1 = not referenced
                        get.append([name, {"t": "present"} if cond[1].endswith("EXACT") else None])
            else:
                name = re.search(r'b\.Get\("([^"]*)"\)', body).group(1)
                want = re.search(r's != "([^"]*)"', body).group(1)
                get = [[name, {"t": "string", "v": want}]]
            gw = local["globalWordList"]
            end = line0 + body.count("\n")
            cases.append({"name": tname, "lines": "%d-%d" % (line0, end), "global": gw, "message": msg, "get": get})
    finally:
        NAMED.clear()
        NAMED.update(saved)
    return {"source": "mixer/pkg/attribute/bag_test.go: each case is a CompressedAttributes message (dictionary "
                      "indices as in the test), the global word list, and the ProtoBag.Get results the test "
                      "asserts ({\"t\": \"present\"}: found). Field maps are [[key, value], ...]; timestamps "
                      "[sec, nsec]; bytes hex.", "cases": cases}


def extract_manifest(ref):
    path = os.path.join(ref, "mixer/testdata/config/attributes.yaml")
    attrs = {}
    name = None
    for line in open(path, encoding="utf-8"):
        m = re.match(r"^\s+([A-Za-z0-9_.]+):\s*$", line)
        if m:
            name = m.group(1)
            continue
        m = re.match(r"^\s+valueType:\s*([A-Z_0-9]+)", line)
        if m and name:
            attrs[name] = m.group(1)
            name = None
    return {"source": "mixer/testdata/config/attributes.yaml", "attributes": attrs}


def extract_checker(ref):
    """mixer/pkg/il/evaluator/checker_test.go: TestTypeCheck (:26-80, the attribute finder and
    expression -> value type or error fragment) and TestAssertType (:82-111, expression + expected
    type -> error fragment, "" = no error)."""
    src = open(os.path.join(ref, "mixer/pkg/il/evaluator/checker_test.go"), encoding="utf-8").read()
    out = {"source": "mixer/pkg/il/evaluator/checker_test.go:26-111"}
    for func, key in (("TestTypeCheck", "type_check"), ("TestAssertType", "assert_type")):
        m = re.search(r"func %s\(t \*testing.T\) \{\s*af := newAF\(\[\]\*ad\{" % func, src)
        attrs = {}
        for _, e in gosrc.Parser(src, m.end() - 1).parse_composite("[]*ad")[2]:
            attrs[conv(e[2][0][1])["v"]] = conv(e[2][1][1])["v"]
        rows = [[conv(v)["v"] for _, v in e[2]] for _, e in _struct_table(src, func)]
        out[key] = {"attrs": attrs, "rows": rows}
    return out


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    outs = {
        "ilt_tests.json": extract_ilt(ref),
        "expr_parse.json": extract_parse(ref),
        "manifest_testdata.json": extract_manifest(ref),
        "il_interpreter.json": extract_interpreter(ref),
        "il_read.json": extract_read(ref),
        "expr_checks.json": extract_expr_checks(ref),
        "externs_kat.json": extract_externs(ref),
        "list_cases.json": extract_lists(ref),
        "resolver_cases.json": extract_resolver(ref),
        "memquota_cases.json": extract_memquota(ref),
        "protobag_cases.json": extract_protobag(ref),
        "checker_cases.json": extract_checker(ref),
    }
    for name, data in outs.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(data, f, indent=1, sort_keys=True)
            f.write("\n")
        print("wrote", name)


if __name__ == "__main__":
    main()
