"""Debug helper: C2 small, print mismatching pairs (got vs oracle) with the request's columns."""
import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "oracle")]
import numpy as np
import oracle
from istio_amd import workloads as W
from istio_amd.engine import Engine, bits_to_codes, load_library
if os.environ.get("MXP_LIB"):
    load_library(os.environ["MXP_LIB"])

if os.environ.get("PRE_C1"):
    m1, r1, b1 = W.c1_workload(512)
    e1 = Engine(0)
    e1.set_vocabulary(m1)
    e1.compile(r1)
    e1.eval_batch(b1)
    del e1
manifest, rules, batch = W.c2_workload(n_rules=int(sys.argv[1]) if len(sys.argv) > 1 else 300, n_requests=int(sys.argv[2]) if len(sys.argv) > 2 else 3000)
eng = Engine(0)
eng.set_vocabulary(manifest)
eng.compile(rules)
print(eng.ruleset_info())
m, e = eng.eval_batch(batch)
got = bits_to_codes(m, e, len(rules))
want = oracle.oracle_matrix(oracle.OracleEvaluator(manifest), rules, batch, threads=8)
want = np.where(want >= 2, 2, want)
bad = np.argwhere(got != want)
print("mismatches", len(bad), "got-true", int(((got == 1) & (want != 1)).sum()), "missed-true",
      int(((got != 1) & (want == 1)).sum()), "got-err", int(((got == 2) & (want != 2)).sum()),
      "missed-err", int(((got != 2) & (want == 2)).sum()))
for q, r in bad[:8]:
    print(q, r, "got", got[q, r], "want", want[q, r], rules[r])
    print("   ", {k: batch.get(int(q), k) for k in ("destination.service", "request.path", "source.ip")})
