"""ORACLE (test infrastructure only) -- restatement of Mixer's runtime.resolver rule selection.

Follows mixer/pkg/runtime/resolver.go:
  Resolve          :110-168  default-namespace rules, then the destination namespace's rules (when
                             different); any error -> (nil, err)
  destAndNamespace :180-199  identity attribute absent -> "not found" error; not a string -> "must
                             be string" error; ns = strings.SplitN(dest, ".", 3)[1] if present
  filterActions    :202-238  tcp := attrs.Get("context.protocol") == "tcp"; per rule in order: skip
                             without an action for the variety; skip when tcp != rule IsTCP; empty
                             match selects; EvalPredicate error -> return the error; true selects.
Predicate results come from the oracle interpreter's pair codes (oracle_matrix); evaluation has no
side effects, so reading a precomputed matrix in resolution order is equivalent.
"""
from __future__ import annotations

OK, NO_IDENTITY, BAD_IDENTITY, PRED_ERROR = 0, 1, 2, 3


def namespace_of(dest: str) -> str:
    parts = dest.split(".", 2)  # strings.SplitN(dest, ".", 3)
    return parts[1] if len(parts) > 1 else ""


def resolve(batch, codes, rule_ns, variety_mask, is_tcp, empty_match, identity_attr, default_ns, variety,
            trace=False):
    """-> list of (status, err_rule or None, [selected rule ids]) per request; with trace, a fourth
    item: the attribute names Resolve itself reads (identity, context.protocol) and the rules whose
    predicate it evaluates, in order (the reads behind ReferencedAttributes)."""
    by_ns = {}
    for r, ns in enumerate(rule_ns):
        by_ns.setdefault(ns, []).append(r)
    out = []
    for q in range(batch.n):
        v, found = batch.get(q, identity_attr)
        if not found:
            out.append((NO_IDENTITY, None, []) + (([identity_attr], []),) * trace)
            continue
        if not isinstance(v, str):
            out.append((BAD_IDENTITY, None, []) + (([identity_attr], []),) * trace)
            continue
        ns = namespace_of(v)
        arr = []
        if default_ns in by_ns:
            arr.append(by_ns[default_ns])
        if default_ns != ns and ns in by_ns:
            arr.append(by_ns[ns])
        p, pf = batch.get(q, "context.protocol")
        tcp = pf and isinstance(p, str) and p == "tcp"
        sel, err, evald = [], None, []
        for rules in arr:
            for r in rules:
                if not (variety_mask[r] >> variety) & 1:
                    continue
                if bool(is_tcp[r]) != tcp:
                    continue
                if not empty_match[r]:
                    evald.append(r)
                    c = int(codes[q, r])
                    if c >= 2:
                        err = r
                        break
                    if c != 1:
                        continue
                sel.append(r)
            if err is not None:
                break
        res = (PRED_ERROR, err, []) if err is not None else (OK, None, sel)
        out.append(res + (([identity_attr, "context.protocol"], evald),) * trace)
    return out


def resolve_referenced(evaluator, rules, batch, q, traced):
    """FakeBag-form referenced list of one Resolve: its own Gets plus the evaluated predicates'."""
    import oracle
    names, evald = traced
    got = {n.encode() for n in names}
    got.update(oracle.oracle_referenced(evaluator, [rules[r] for r in evald], batch, q))
    return sorted(got)
