"""The oracle (CPU restatement) against the reference's own golden table and parse KATs.

Pins oracle/goexpr.py + oracle/ilcompile.py + oracle/il_interp.c to
  mixer/pkg/il/testing/tests.go:37-2258 (expressions, IL text, bags, results, errors) and
  mixer/pkg/expr/expr_test.go:27-76 (parse -> postfix forms).
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
    if isinstance(expected, bool) or isinstance(actual, bool):
        return type(expected) is type(actual) and expected == actual
    return type(expected) is type(actual) and expected == actual


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


@pytest.mark.parametrize("src,frag", [
    ("*a != b", "unexpected expression"), ("a = bc", "unable to parse"), ("3 = 10", "unable to parse"),
    ("(a.c).d == 300", "unexpected expression"), ("substring(*a, 20) == 12", "unexpected expression"),
    ("(*a == 20) && 12", "unexpected expression"), ("!*a", "unexpected expression"),
    ("request.headers[*a] == 200", "unexpected expression"), ("atr == 'aaa'", "unable to parse"),
    ("c().e.d()", "unexpected expression"), ("foo{}", "unexpected expression"),
    ("foo{}.bar", "unexpected expression"), ("foo{}.bar()", "unexpected expression"),
    ("(foo{}).bar()", "unexpected expression"), ("a().b", "unexpected expression"),
])
def test_bad_parse(src, frag):
    """mixer/pkg/expr/expr_test.go:190-246."""
    with pytest.raises(goexpr.ParseError) as ei:
        goexpr.parse(src)
    assert frag in str(ei.value)


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
