"""Referenced attributes at scale: mxp_eval_refs end to end (host batch in, per-request referenced
sets out: pack + upload, the *_refs kernels, record download, host assembly) against plain
mxp_eval_batch on the same batch.  One JSON line per workload."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from istio_amd import workloads as W  # noqa: E402
from istio_amd.engine import Engine  # noqa: E402

n_req = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
for wl in sys.argv[1].split(","):
    if wl == "c4":
        manifest, rules, batch = W.c4_workload(n_rules=10000, n_requests=n_req, seed=4)
    else:
        manifest, rules, batch = W.c2_workload(n_rules=10000, n_requests=n_req, seed=2)
    eng = Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    eng.eval_batch(batch)
    t0 = time.perf_counter()
    eng.eval_batch(batch)
    t_eval = time.perf_counter() - t0
    eng.eval_refs_raw(batch)
    t0 = time.perf_counter()
    off, ents = eng.eval_refs_raw(batch)
    t_refs = time.perf_counter() - t0
    per = np.diff(off)
    print(json.dumps({"workload": wl, "rules": len(rules), "requests": batch.n,
                      "eval_batch_s": t_eval, "eval_refs_s": t_refs,
                      "refs_per_request_mean": float(per.mean()), "refs_per_request_max": int(per.max()),
                      "requests_per_s_with_refs": batch.n / t_refs}), flush=True)
