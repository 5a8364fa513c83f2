"""The product's C++ front end / IL code generator (libmxp, host-only engine) against the golden
table and against the oracle on generated rule sets; and the lowering's coverage."""
import json
import os

import numpy as np
import pytest

import goexpr
import ilcompile
from istio_amd import workloads as W

HERE = os.path.dirname(os.path.abspath(__file__))
ROWS = json.load(open(os.path.join(HERE, "golden", "ilt_tests.json")))


@pytest.fixture(scope="module")
def Engine(libmxp):
    from istio_amd.engine import Engine
    return Engine


def test_golden_compile(Engine):
    mism = []
    for row in ROWS["rows"]:
        if not row.get("E") or "Fns" in row:
            continue
        e = Engine(-1)
        e.set_vocabulary(ROWS["manifests"][row.get("conf", "defaultAttrs")])
        st = e.compile([row["E"]])[0]
        if "CompileErr" in row:
            if st == 0 or e.rule_error(0) != row["CompileErr"]:
                mism.append((row["index"], e.rule_error(0)))
            continue
        if st != 0:
            mism.append((row["index"], st, e.rule_error(0)))
            continue
        if "IL" in row and e.rule_il_text(0).strip() != row["IL"].strip():
            mism.append((row["index"], e.rule_il_text(0)))
    assert not mism


def _oracle_compile(manifest, rule):
    attrs = {k: goexpr.VT[v] for k, v in manifest.items()}
    try:
        p, _ = ilcompile.compile_expr(rule, attrs)
        return ilcompile.write_text(p), None
    except Exception as e:  # noqa: BLE001 -- every reference error class is compared by text
        return None, str(e)


@pytest.mark.parametrize("which", ["c1", "c2", "fuzz"])
def test_matches_oracle_codegen(Engine, which):
    if which == "c1":
        manifest, rules, _ = W.c1_workload(10)
    elif which == "c2":
        manifest, rules = W.TESTDATA_MANIFEST, W.c2_rules(500)[0]
    else:
        manifest, rules = W.DEFAULT_TEST_MANIFEST, W.fuzz_rules(1500, seed=11, depth=3)
    e = Engine(-1)
    e.set_vocabulary(manifest)
    st = e.compile(rules)
    for i, r in enumerate(rules):
        text, err = _oracle_compile(manifest, r)
        if err is not None:
            assert st[i] != 0 and e.rule_error(i) == err, r
        else:
            assert st[i] in (0, 5), (r, e.rule_error(i))
            assert e.rule_il_text(i) == text, r
    # every generated rule without a regexp lowers to the GPU bytecode
    unsupported = [rules[i] for i in np.where(st == 5)[0]]
    assert not unsupported, unsupported[:3]


def test_compiler_sessions(Engine):
    """compiler_test.go:30-136 runs every tests.go expression through a compile *session*: once
    (TestCompiler_SingleExpressionSession, IL as Compile writes it) and twice into the same program
    (TestCompiler_DoubleExpressionSession, both functions evaluate alike).  The engine's session is a
    rule set: every expression of the golden table compiled twice in ONE rule set, beside the other
    rows, keeps its own IL, its own compile error text, and identical statuses for both copies."""
    by_conf = {}
    for row in ROWS["rows"]:
        if row.get("E") and "Fns" not in row:
            by_conf.setdefault(row.get("conf", "defaultAttrs"), []).append(row)
    checked = 0
    for conf, rows in by_conf.items():
        e = Engine(-1)
        e.set_vocabulary(ROWS["manifests"][conf])
        exprs = [r["E"] for r in rows for _ in (0, 1)]  # each expression twice, in table order
        st = e.compile(exprs)
        for k, row in enumerate(rows):
            a, b = 2 * k, 2 * k + 1
            assert st[a] == st[b], row["E"]
            if "CompileErr" in row:
                assert st[a] != 0 and e.rule_error(a) == e.rule_error(b) == row["CompileErr"], row["E"]
                continue
            assert st[a] == 0, (row["E"], e.rule_error(a))
            assert e.rule_il_text(a) == e.rule_il_text(b)
            if "IL" in row:
                assert e.rule_il_text(a).strip() == row["IL"].strip(), row["E"]
            checked += 1
    assert checked > 150


def test_reference_limit_rules_compile(Engine):
    """Rules at the reference VM's limits are lowered, not refused (MXP_RULE_UNSUPPORTED = 5): long
    chains up to the heap limit (static per-path counts, or the VM_HEAP count register when paths
    merge with different counts), `|` chains past the 64-word stack, right-nested comparisons
    (coloured onto the deep kernels' 64 registers), run-time regexp patterns of every provenance."""
    e = Engine(-1)
    e.set_vocabulary(W.DEFAULT_TEST_MANIFEST)
    rules = W.hard_fuzz_rules(800, seed=21) + W.fuzz_rules(800, seed=22, depth=4)
    rules.append(" | ".join('(as == "a%d")' % i for i in range(70)))  # straight line: static heap count
    st = e.compile(rules)
    assert (st != 5).all(), [(rules[i][:60], e.rule_error(i)) for i in np.where(st == 5)[0][:3]]
    vm = {i: e.rule_vm_text(i) for i in range(len(rules)) if st[i] == 0}
    assert any(" heap " in t for t in vm.values())  # the dynamic heap count
    assert any("y=15 " in t and " err " in t for t in vm.values())  # a static "heap overflow" (ERR_HEAP)
    assert any("y=14 " in t and " err " in t for t in vm.values())  # "stack overflow" (ERR_OVERFLOW)
    assert any(" regexd " in t for t in vm.values())
    # registers: the hot kernels' 8 unless the rule is deep (up to 64)
    regs = [max(int(tok[2:]) for line in t.splitlines() for tok in line.split()[2:5]) for t in vm.values()]
    assert max(regs) >= 8 and max(regs) < 64
    # ordinary rules are lowered exactly as before: no heap register, registers from 0 by depth
    plain = Engine(-1)
    plain.set_vocabulary(W.DEFAULT_TEST_MANIFEST)
    assert (plain.compile(['as == "a" && bs.startsWith("b")']) == 0).all()
    assert " heap " not in plain.rule_vm_text(0)


def test_heap_panic_after_extern_in_oracle():
    """The oracle's heap: an ip() return takes slot 63 without the check (extern.go:232-237); the next
    checked push writes heap[64]: Go's "index out of range" panic, not "heap overflow"."""
    import oracle
    from istio_amd.bags import BagBatch
    rule = " || ".join('as == "x%d"' % i for i in range(62)) + ' || ip(as) == ip("1.2.3.4") || bs == "abc"'
    batch = BagBatch.from_bags([{"as": "1.2.3.4", "bs": "abc"}, {"as": "nope", "bs": "abc"}, {"as": "x3"}],
                               names=list(W.DEFAULT_TEST_MANIFEST))
    ev = oracle.OracleEvaluator(W.DEFAULT_TEST_MANIFEST)
    assert ev.eval_predicate(rule, batch, 0) == ("panic", "runtime error: index out of range")
    assert ev.eval_predicate(rule, batch, 1) == ("error", "could not convert nope to IP_ADDRESS")
    assert ev.eval_predicate(rule, batch, 2) == ("ok", True)
    chain = " || ".join('as == "x%d"' % i for i in range(70))
    assert ev.eval_predicate(chain, batch, 1) == ("error", "heap overflow")
    assert ev.eval_predicate(chain, batch, 2) == ("ok", True)


def deep_continuation_rules(n=64):
    """`as == K && <constant-free continuation with more than 8 values live>`: guard-led rules whose
    continuation needs the deep kernels' registers (such a continuation must never become
    an index template, whose kernels have MXP_VM_MAXREG registers)."""
    deep = "(" + "bb == (" * 12 + "bb" + ")" * 12 + ")"
    return ['as == "x%d" && %s' % (i, deep) for i in range(n)] + ['as == "y%d" && bs == "b" && %s' % (i, deep)
                                                                    for i in range(8)]


def test_deep_continuations_are_not_indexed(Engine):
    e = Engine(-1)
    e.set_vocabulary(W.DEFAULT_TEST_MANIFEST)
    rules = deep_continuation_rules()
    assert (e.compile(rules) == 0).all()
    info = e.ruleset_info()
    assert info["guarded"] == len(rules)
    assert info["templated"] == 0 and info["indexed"] == 0, info
    # a shallow continuation of the same shape is still templated and indexed
    s = Engine(-1)
    s.set_vocabulary(W.DEFAULT_TEST_MANIFEST)
    assert (s.compile(['as == "x%d" && (bb == (bb == bb))' % i for i in range(64)]) == 0).all()
    assert s.ruleset_info()["indexed"] == 64
