"""The C-ABI library loads and exports every entry point include/*.h declares (no GPU needed)."""
import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def declared_functions():
    names = set()
    for h in os.listdir(os.path.join(ROOT, "include")):
        if h.endswith(".h"):
            src = open(os.path.join(ROOT, "include", h)).read()
            names |= set(re.findall(r"^\s*(?:[A-Za-z_][A-Za-z0-9_ \*]*?[\s\*])(mxp_[a-z0-9_]+)\s*\(", src, re.M))
    return names


def test_exports_all_declared_symbols(libmxp):
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(libmxp, n)]
    assert not missing


def test_python_mirror_binds_every_symbol(libmxp):
    from istio_amd.engine import SIGNATURES
    assert declared_functions() == set(SIGNATURES)


def test_host_only_engine_refuses_eval(libmxp):
    from istio_amd.engine import Engine, MxpError
    from istio_amd.bags import BagBatch
    e = Engine(-1)
    e.set_vocabulary({"a": "INT64"})
    assert list(e.compile(["a == 2"])) == [0]
    try:
        e.eval_batch(BagBatch.from_bags([{"a": 2}]))
    except MxpError as ex:
        assert "host-only" in str(ex)
    else:
        raise AssertionError("host-only engine evaluated")


def test_gfx950_code_object(libmxp):
    data = open(os.path.join(ROOT, "istio_amd", "libmxp.so"), "rb").read()
    assert b"gfx950" in data


def test_ruleset_columns(libmxp):
    """mxp_ruleset_columns: the attributes a rule set reads (columns, then map attributes of
    map["key"] reads), then the resolver's identity and context.protocol (host-only engine)."""
    import numpy as np
    from istio_amd.engine import Engine
    eng = Engine(-1)
    assert eng.read_attributes() == []
    eng.set_vocabulary({"a": "STRING", "b": "INT64", "m": "STRING_MAP", "destination.service": "STRING",
                        "context.protocol": "STRING"})
    eng.compile(['a == "x" && b == 2', 'm["k"] == a', 'a.startsWith("y")'])
    assert eng.read_attributes() == ["a", "b", "m"]
    eng.set_resolver("destination.service", "default", ["default"] * 3, np.ones(3, np.uint32), np.zeros(3, np.uint8),
                     np.zeros(3, np.uint8))
    assert eng.read_attributes() == ["a", "b", "m", "destination.service", "context.protocol"]


def test_vocabulary_finder(libmxp):
    """mxp_vocab_set_finder (ChangeVocabulary(finder), runtime/controller.go:100-102): names are
    asked for on first use; the rule set compiles exactly as with the whole manifest given up front
    (statuses, IL, error texts, VM code), unknown names give the reference's type-check error, and
    vocabulary positions (mxp_attr_ref.attr) name the attributes through mxp_vocab_name."""
    from istio_amd import workloads as W
    from istio_amd.engine import Engine
    manifest = dict(W.DEFAULT_TEST_MANIFEST)
    asked = []

    def get_attribute(name):
        asked.append(name)
        return manifest.get(name)
    rules = W.fuzz_rules(300, seed=5, depth=3) + W.hard_fuzz_rules(50, seed=6) + ["nope == 2", 'as == "x"']
    a, b = Engine(-1), Engine(-1)
    a.set_vocabulary(manifest)
    b.set_vocabulary_finder(get_attribute)
    sa, sb = a.compile(rules), b.compile(rules)
    assert list(sa) == list(sb)
    for i in range(len(rules)):
        assert a.rule_error(i) == b.rule_error(i)
        if sa[i] == 0:
            assert a.rule_il_text(i) == b.rule_il_text(i)
    assert "nope" in asked and len(asked) == len(set(asked))  # each name asked once
    known = [n for n in asked if n in manifest]
    assert [b.vocab_name(p) for p in range(len(known))] == known  # positions in the order asked


def test_go_binding_calls_declared_symbols():
    """Every C.mxp_* call and C.MXP_* constant in INTEGRATION.md's Go text is declared by
    include/*.h, and the binding asserts the reference interfaces it implements."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    go = "\n".join(re.findall(r"```go\n(.*?)```", text, re.S))
    calls = set(re.findall(r"\bC\.(mxp_[a-z0-9_]+)\s*\(", go))
    assert calls and not calls - declared_functions(), calls - declared_functions()
    hdr = "".join(open(os.path.join(ROOT, "include", h)).read() for h in os.listdir(os.path.join(ROOT, "include")))
    consts = set(re.findall(r"\bC\.(MXP_[A-Z0-9_]+)\b", go))
    assert not [c for c in consts if not re.search(r"\b%s\b" % c, hdr)]
    for iface in ("var _ expr.Evaluator = (*Batcher)(nil)",
                  "var _ runtime.VocabularyChangeListener = (*Batcher)(nil)",
                  "var _ Resolver = (*mxpResolver)(nil)", "var _ Actions = (*actions)(nil)",
                  "var _ list = (*gpuList)(nil)", "var _ listentry.Handler = (*gpuHandler)(nil)",
                  "var _ listentry.BagHandler = (*gpuHandler)(nil)",
                  "var _ expr.TypeChecker = (*TypeChecker)(nil)", "var _ compiled.Expression = Expression{}"):
        assert iface in go, iface
    # the reference's per-Resolve observations (resolver.go:123-138, monitor.go:51-89) in the drop-in
    for obs in ("resolveCounter.With(lbls).Inc()", "resolveDuration.With(lbls).Observe(",
                "resolveRules.With(lbls).Observe(float64(nselected))", "resolveActions.With(lbls).Observe(float64(raLen))",
                "prometheus.Labels{targetStr: target, errorStr: strconv.FormatBool(err != nil)}"):
        assert obs in go, obs
    # the device group: one process over every GPU, its all-reduce and owner-routed memquota bound
    for name in ("mxp_group_create", "mxp_group_ruleset_compile", "mxp_group_resolver_set", "mxp_group_resolve_batch",
                 "mxp_group_reduce", "mxp_group_counters", "mxp_group_key_owners", "mxp_group_quota_create",
                 "mxp_group_quota_alloc", "mxp_group_pair_error", "mxp_group_vocab_set_finder"):
        assert name in calls, name
    # the list adapter's device calls (mxp_list*) are all bound, each with the header's arity
    hdr_decl = {m.group(1): m.group(2) for m in re.finditer(r"\b(mxp_list[a-z_]*)\(([^;]*?)\);", hdr, re.S)}
    for name in ("mxp_list_create", "mxp_list_check", "mxp_listentry_check", "mxp_list_entries", "mxp_list_destroy"):
        assert name in calls, name
    for m in re.finditer(r"\bC\.(mxp_list[a-z_]*)\(", go):
        depth, n_args, i = 1, 1, m.end()
        if go[i] == ")":
            n_args = 0
        while depth:
            ch = go[i]
            depth += ch in "(["
            depth -= ch in ")]"
            n_args += ch == "," and depth == 1
            i += 1
        assert n_args == hdr_decl[m.group(1)].count(",") + 1, (m.group(1), go[m.end():i])
