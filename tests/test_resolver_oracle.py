"""The resolver restatement (oracle/resolver.py) against the reference's own resolver table
(mixer/pkg/runtime/resolver_test.go:38-145, transcribed into tests/golden/resolver_cases.json)."""
import json
import os

import numpy as np
import pytest

import resolver as oracle_resolver
from istio_amd.bags import BagBatch

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "resolver_cases.json")))


def case_inputs(case):
    rule_ns, lengths = [], []
    for ns, length in case["rules"]:
        rule_ns.append(ns)
        lengths.append(length)
    # the reference builds map[ns][]*Rule, so rules of a namespace are contiguous in resolution order
    order = sorted(range(len(rule_ns)), key=lambda i: (rule_ns[i], i))
    rule_ns = [rule_ns[i] for i in order]
    lengths = [lengths[i] for i in order]
    bag = dict(case["bag"])
    batch = BagBatch.from_bags([bag], names=["destination.service", "context.protocol"])
    return rule_ns, lengths, batch


@pytest.mark.parametrize("case", CASES["cases"], ids=[c["desc"] for c in CASES["cases"]])
def test_reference_resolver_table(case):
    rule_ns, lengths, batch = case_inputs(case)
    n = len(rule_ns)
    code = 2 if case.get("selectError") else (0 if case.get("selectReject") else 1)
    codes = np.full((1, max(n, 1)), code, dtype=np.uint8)
    (status, err_rule, sel), = oracle_resolver.resolve(
        batch, codes, rule_ns, [1] * n, [0] * n, [0] * n, CASES["identity_attr"], CASES["default_ns"],
        case.get("callVariety", 0))
    if "err" in case:
        want = oracle_resolver.NO_IDENTITY if "identity" in case["err"] else oracle_resolver.PRED_ERROR
        assert status == want
        return
    assert status == oracle_resolver.OK
    assert sum(lengths[r] for r in sel) == case["nactions"]


def test_namespace_split():
    assert oracle_resolver.namespace_of("a.b.c.d") == "b"
    assert oracle_resolver.namespace_of("a.b") == "b"
    assert oracle_resolver.namespace_of("a") == ""
    assert oracle_resolver.namespace_of(".x") == "x"
