#!/usr/bin/env python3
"""Extract the reference's Go test tables into JSON fixtures (data only).

Run in the build container, where the read-only reference is mounted:

    python tests/golden/make_fixtures.py [/root/reference]

Outputs (committed):
  tests/golden/ilt_tests.json      <- mixer/pkg/il/testing/tests.go:37-2258 (TestData) and the two
                                      attribute manifests at tests.go:2342-2489
  tests/golden/expr_parse.json     <- mixer/pkg/expr/expr_test.go:27-76 (TestGoodParse postfix forms)
  tests/golden/manifest_testdata.json <- mixer/testdata/config/attributes.yaml (names + ValueType)

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
}


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
        if name.startswith("descriptor."):
            return {"t": "valuetype", "v": name.split(".", 1)[1]}
        return {"t": "ident", "v": name}
    if kind == "concat":
        a, b = conv(node[1]), conv(node[2])
        assert a["t"] == "string" and b["t"] == "string"
        return {"t": "string", "v": a["v"] + b["v"]}
    if kind == "call":
        name, args = node[1], node[2]
        if name == "int64":
            a = conv(args[0])
            return {"t": "int64", "v": a["v"]}
        if name == "float64":
            a = args[0]
            return {"t": "float64", "v": repr(float(a[1]))}
        if name == "net.ParseIP":
            return {"t": "bytes", "v": parse_ipv4_16(conv(args[0])["v"])}
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
        return {"t": "composite", "typ": typ, "v": [[None if k is None else conv(k), conv(v)] for k, v in elems]}
    if kind == "func":
        return {"t": "func", "v": node[1]}
    if kind == "neg":
        a = conv(node[1])
        return {"t": a["t"], "v": "-" + a["v"]}
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
    m = re.search(r"func TestGoodParse\(t \*testing.T\) \{\s*tests := \[\]struct \{[^}]*\}\{", src)
    p = gosrc.Parser(src, m.end() - 1)
    lit = p.parse_composite("[]struct")
    cases = [[conv(e[1][2][0][1])["v"], conv(e[1][2][1][1])["v"]] for e in lit[2]]
    return {"source": "mixer/pkg/expr/expr_test.go:27-76", "cases": cases}


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


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    outs = {
        "ilt_tests.json": extract_ilt(ref),
        "expr_parse.json": extract_parse(ref),
        "manifest_testdata.json": extract_manifest(ref),
    }
    for name, data in outs.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(data, f, indent=1, sort_keys=True)
            f.write("\n")
        print("wrote", name)


if __name__ == "__main__":
    main()
