"""Diagnose: resolve (error-bitmap mode) error bits without records on the resolver workload."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa
import torch  # noqa
from istio_amd import workloads as W  # noqa
import istio_amd.engine as mxp  # noqa

mode = sys.argv[1] if len(sys.argv) > 1 else "bitmap"
if mode == "bitmap":
    os.environ["MXP_DEBUG_FLAGS"] = "268435456"
manifest, rules, conf, batch = W.resolver_workload(n_rules=600, n_requests=3000, seed=21)
eng = mxp.Engine(0)
eng.set_vocabulary(manifest)
eng.compile(rules)
eng.set_resolver(conf["identity_attr"], conf["default_ns"], conf["rule_ns"], conf["variety_mask"], conf["is_tcp"],
                 conf["empty_match"])
print("ruleset", eng.ruleset_info())
for variety in (0, 2, 3):
    status, err_rule, sel = eng.resolve(batch, variety)
    bad = []
    for q in np.nonzero(status == 3)[0]:
        t = eng.pair_error(int(q), int(err_rule[q]))
        if not t:
            bad.append((int(q), int(err_rule[q])))
    print("variety", variety, "failing", int((status == 3).sum()), "without text", len(bad), bad[:5])
    for q, r in bad[:3]:
        print("  rule", r, rules[r])
        print("  vm", eng.rule_vm_text(r).replace("\n", " | ")[:400])
        print("  bag", {k: batch.get(q, k) for k in batch.names})
# the same batch through eval_batch
m, e = eng.eval_batch(batch)
codes = mxp.bits_to_codes(m, e, len(rules))
errs = np.argwhere(codes == 2)
no = [(int(q), int(r)) for q, r in errs if not eng.pair_error(int(q), int(r))]
print("eval_batch error pairs", len(errs), "without text", len(no), no[:5])
