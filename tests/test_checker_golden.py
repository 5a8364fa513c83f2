"""expr.TypeChecker pinned by the reference's own table: mixer/pkg/il/evaluator/checker_test.go
TestTypeCheck (:26-80) and TestAssertType (:82-111), extracted as data into
tests/golden/checker_cases.json by make_fixtures.py.  Checked on both sides: the oracle's EvalType
restatement (oracle/goexpr.py) and the product's front end (engine.TypeChecker over
mxp_ruleset_compile / mxp_rule_types on a host-only engine)."""
import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import goexpr  # noqa: E402

CASES = json.load(open(os.path.join(HERE, "golden", "checker_cases.json")))
TC, AT = CASES["type_check"], CASES["assert_type"]


def test_fixture_shape():
    assert len(TC["rows"]) == 16 and len(AT["rows"]) == 3


@pytest.fixture(scope="module")
def checker(libmxp):
    from istio_amd.engine import TypeChecker
    return TypeChecker()


def _oracle_eval_type(src, attrs):
    """checker.EvalType (checker.go:29-35) over the oracle restatement."""
    try:
        e = goexpr.parse(src)
    except goexpr.ParseError as err:
        return "VALUE_TYPE_UNSPECIFIED", "failed to parse expression '%s': %s" % (src, err)
    try:
        t = goexpr.eval_type(e, {k: goexpr.VT[v] for k, v in attrs.items()}, goexpr.func_map())
    except goexpr.TypeCheckError as err:
        return "VALUE_TYPE_UNSPECIFIED", str(err)
    return goexpr.vt_name(t), None


@pytest.mark.parametrize("row", TC["rows"], ids=lambda r: r[0])
def test_type_check(checker, row):
    src, want, frag = row
    for t, err in (checker.eval_type(src, TC["attrs"]), _oracle_eval_type(src, TC["attrs"])):
        # (the Go test: an error must contain the fragment, and the type must equal `out` either way)
        if frag or err is not None:
            assert err is not None and frag in err, (src, err)
        assert t == want, (src, t)


@pytest.mark.parametrize("row", AT["rows"], ids=lambda r: r[0])
def test_assert_type(checker, row):
    _, src, expected, frag = row
    err = checker.assert_type(src, AT["attrs"], expected)
    if frag:
        assert err is not None and frag in err, err
    else:
        assert err is None, err
    t, oerr = _oracle_eval_type(src, AT["attrs"])
    if oerr is None and t != expected:
        oerr = "expression '%s' evaluated to type %s, expected type %s" % (src, t, expected)
    assert (oerr is None) == (err is None) and (not frag or frag in oerr)
