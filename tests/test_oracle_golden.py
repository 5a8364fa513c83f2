"""The oracle (CPU restatement) against the reference's own golden table and parse KATs.

Pins oracle/goexpr.py + oracle/ilcompile.py + oracle/il_interp.c to
  mixer/pkg/il/testing/tests.go:37-2258 (expressions, IL text, bags, results, errors),
  mixer/pkg/expr/expr_test.go:27-76 (parse -> postfix forms), :190-246 (bad parses) and :258-333
  (type checks), and mixer/pkg/il/runtime/externs_test.go:24-129 (extern KATs).
"""
import json
import os

import pytest

import goexpr
import ilcompile
import oracle
from istio_amd.bags import BagBatch, from_tagged

HERE = os.path.dirname(os.path.abspath(__file__))
ROWS = json.load(open(os.path.join(HERE, "golden", "ilt_tests.json")))


def fmap_for(row):
    fns = goexpr.extern_metadata()
    for f in row.get("Fns", []):
        fns.append(goexpr.FunctionMetadata(f["Name"], f["Instance"], goexpr.VT[f["TargetType"]],
                                           goexpr.VT[f["ReturnType"]], [goexpr.VT[a] for a in f["ArgumentTypes"]]))
    return goexpr.func_map(fns)


def same_value(expected, actual):
    """ilt.AreEqual (il/testing/util.go:22-32) over the Python Go-value model."""
    if isinstance(expected, bytes):
        return isinstance(actual, bytes) and expected == actual
    # (the product's istio_amd.bags and the oracle's govalue types: compared by type name)
    return type(expected).__name__ == type(actual).__name__ and expected == actual


@pytest.mark.parametrize("row", [r for r in ROWS["rows"] if r.get("E")], ids=lambda r: "%d" % r["index"])
def test_golden_row(row):
    conf = ROWS["manifests"][row.get("conf", "defaultAttrs")]
    ev = oracle.OracleEvaluator(conf, fmap_for(row))
    try:
        prog, _ = ilcompile.compile_expr(row["E"], ev.attrs, ev.fmap)
        cerr = None
    except (goexpr.ParseError, goexpr.TypeCheckError, ilcompile.CompileError) as e:
        prog, cerr = None, str(e)
    if "CompileErr" in row:
        assert cerr == row["CompileErr"]
        return
    assert cerr is None
    if "IL" in row:
        assert ilcompile.write_text(prog).strip() == row["IL"].strip()
    if "Externs" in row:
        return  # custom test-only extern (`reverse`), not part of the product surface
    batch = BagBatch.from_bags([{k: from_tagged(v) for k, v in row.get("I", {}).items()}])
    st, v = ev.eval(row["E"], batch, 0)
    if "Err" in row:
        assert st == "error" and v.startswith(row["Err"])
    else:
        assert st == "ok", v
        assert same_value(from_tagged(row["R"]), v)


@pytest.mark.parametrize("row", [r for r in ROWS["rows"] if r.get("E") and "Referenced" in r],
                         ids=lambda r: "%d" % r["index"])
def test_golden_referenced(row):
    """The oracle's referenced-attribute tracking against the rows' `Referenced` lists
    (FakeBag.ReferencedList, il/testing/fakebag.go:75; checked by evaluator_test.go:73)."""
    conf = ROWS["manifests"][row.get("conf", "defaultAttrs")]
    ev = oracle.OracleEvaluator(conf, fmap_for(row))
    batch = BagBatch.from_bags([{k: from_tagged(v) for k, v in row.get("I", {}).items()}])
    got = [x.decode() for x in oracle.oracle_referenced(ev, [row["E"]], batch, 0)]
    assert got == row["Referenced"]


def test_parse_postfix_forms():
    cases = json.load(open(os.path.join(HERE, "golden", "expr_parse.json")))["cases"]
    assert len(cases) == 29
    for src, post in cases:
        assert str(goexpr.parse(src)) == post


CHECKS = json.load(open(os.path.join(HERE, "golden", "expr_checks.json")))


@pytest.mark.parametrize("src,frag", CHECKS["bad_parse"])
def test_bad_parse(src, frag):
    """mixer/pkg/expr/expr_test.go:190-246 (TestBadParse)."""
    with pytest.raises(goexpr.ParseError) as ei:
        goexpr.parse(src)
    assert frag in str(ei.value)


@pytest.mark.parametrize("case", CHECKS["type_checks"], ids=lambda c: c["s"])
def test_internal_type_check(case):
    """mixer/pkg/expr/expr_test.go:258-333 (TestInternalTypeCheck): FuncMap(fns) holds the intrinsics
    plus the case's functions only; EvalType returns the type or an error containing the fragment."""
    fns = [goexpr.FunctionMetadata(f["Name"], f["Instance"], goexpr.VT[f["TargetType"]], goexpr.VT[f["ReturnType"]],
                                   [goexpr.VT[a] for a in f["ArgumentTypes"]]) for f in case["fns"]]
    attrs = {k: goexpr.VT[v] for k, v in case["attrs"].items()}
    e = goexpr.parse(case["s"])
    try:
        t = goexpr.eval_type(e, attrs, goexpr.func_map(fns))
    except goexpr.TypeCheckError as err:
        assert case["err"] != "__SUCCESS__" and case["err"] in str(err), str(err)
        return
    assert case["err"] == "__SUCCESS__"
    assert t == goexpr.VT[case["ret"]]


def test_duration_and_constants():
    """expr.newConstant (expr.go:123-152) and expr_test.go:160-188."""
    assert goexpr.new_constant('"19ms"', goexpr.STRING).type == goexpr.DURATION
    assert goexpr.new_constant('"0"', goexpr.STRING).type == goexpr.DURATION
    assert goexpr.new_constant('"abc"', goexpr.STRING).type == goexpr.STRING
    assert goexpr.new_constant("3.75", goexpr.DOUBLE).value == 3.75
    assert goexpr.new_constant("1001", goexpr.INT64).value == 1001
    assert goexpr.new_constant("`back quoted`", goexpr.STRING).value == "back quoted"
    assert goexpr.go_parse_duration("1.5h") == 5400 * 10**9
    assert goexpr.go_parse_duration("-1m30s") == -90 * 10**9
    with pytest.raises(ValueError):
        goexpr.go_parse_duration("1")


EXTERNS = json.load(open(os.path.join(HERE, "golden", "externs_kat.json")))["cases"]


def extern_expr(case):
    """The extern KAT as a Mixer expression over attributes s1, s2 (so it runs, not folds)."""
    fn = case["fn"]
    if fn == "ip":
        return "ip(s1)"
    if fn == "timestamp":
        return "timestamp(s1)"
    if fn == "ip_equal":
        return "ip(s1) == ip(s2)"
    if fn == "timestamp_equal":
        return "timestamp(s1) == timestamp(s2)"
    if fn == "match":
        return "match(s1, s2)"
    return "s1.matches(s2)"


def extern_bag(case):
    a = case["args"]
    return {"s1": a[0], "s2": a[1] if len(a) > 1 else a[0]}


@pytest.mark.parametrize("case", EXTERNS, ids=lambda c: "%s%s" % (c["fn"], c["args"]))
def test_extern_kat(case):
    import datetime
    from govalue import GoTime
    ev = oracle.OracleEvaluator({"s1": "STRING", "s2": "STRING"})
    batch = BagBatch.from_bags([extern_bag(case)])
    st, v = ev.eval(extern_expr(case), batch, 0)
    if case.get("err"):
        assert st == "error", v
        return
    assert st == "ok", v
    if "want_fields" in case:
        assert isinstance(v, GoTime)
        t = datetime.datetime.fromtimestamp(v.sec, datetime.timezone.utc)
        assert [t.year, t.month, t.day, t.hour, t.minute] == case["want_fields"]
    elif isinstance(case["want"], dict):
        assert same_value(from_tagged(case["want"]), v)
    else:
        assert v is case["want"]
