"""Steady-state evaluation rate: K evaluations enqueued back to back on one stream (no per-evaluation
synchronisation, as the bench's timed loop runs them), for each engine setting in turn, alternated
over repetitions.  Prints host enqueue time and wall time per evaluation.
    usage: steady.py c2|c4 "" "MXP_X=1" ..."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from istio_amd import workloads as W  # noqa: E402
from istio_amd.engine import Engine  # noqa: E402

wl, settings = sys.argv[1], sys.argv[2:] or [""]
if wl == "c4":
    manifest, rules, batch = W.c4_workload(n_rules=10000, n_requests=1 << 20, seed=4)
else:
    manifest, rules, batch = W.c2_workload(n_rules=10000, n_requests=1 << 20, seed=2)
Wd = (len(rules) + 31) // 32
dm = torch.empty((Wd, batch.n), dtype=torch.int32, device="cuda:0")
hits = torch.zeros(len(rules), dtype=torch.int64, device="cuda:0")
flags = torch.empty(batch.n, dtype=torch.uint8, device="cuda:0")
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
K = 50
res = {x: [] for x in settings}
for rep in range(3):
    for st in settings:
        saved = dict(os.environ)
        for kv in st.split(","):
            if kv:
                k, v = kv.split("=")
                os.environ[k] = v
        eng = Engine(0)
        os.environ.clear()
        os.environ.update(saved)
        eng.set_vocabulary(manifest)
        eng.compile(rules)
        db = eng.upload(batch)
        for _ in range(5):
            db.eval_compact(dm.data_ptr(), flags.data_ptr(), hits.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            db.eval_compact(dm.data_ptr(), flags.data_ptr(), hits.data_ptr(), s.cuda_stream)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res[st].append(((t1 - t0) / K * 1e3, (t2 - t0) / K * 1e3))
        db.free()
        del eng
for st, v in res.items():
    print("%s %-24s enqueue ms/eval %s  wall ms/eval %s  median wall %.4f" % (
        wl, st or "(default)", ["%.3f" % a for a, _ in v], ["%.4f" % b for _, b in v], np.median([b for _, b in v])), flush=True)
