"""Sweep mxp_set_pipeline settings on one workload: ms per evaluation (HIP events on the stream)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from istio_amd import workloads as W  # noqa: E402
from istio_amd.engine import Engine  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
if wl == "c4":
    manifest, rules, batch = W.c4_workload(n_rules=10000, n_requests=1 << 20, seed=4)
else:
    manifest, rules, batch = W.c2_workload(n_rules=10000, n_requests=1 << 20, seed=2)
eng = Engine(0)
eng.set_vocabulary(manifest)
eng.compile(rules)
db = eng.upload(batch)
Wd = (len(rules) + 31) // 32
dm = torch.empty((Wd, batch.n), dtype=torch.int32, device="cuda:0")
de = torch.empty_like(dm)
hits = torch.zeros(len(rules), dtype=torch.int64, device="cuda:0")
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
for setting in [(1 << 30, 1), (1 << 19, 2), (1 << 18, 4), (1 << 17, 8), (1 << 18, 2), (1 << 30, 1)]:
    eng.set_pipeline(*setting)
    for _ in range(3):
        db.eval_hits(dm.data_ptr(), de.data_ptr(), hits.data_ptr(), s.cuda_stream)
    ts = []
    for _ in range(10):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        db.eval_hits(dm.data_ptr(), de.data_ptr(), hits.data_ptr(), s.cuda_stream)
        b.record(s)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    print(wl, setting, "ms median %.3f min %.3f" % (np.median(ts), np.min(ts)), flush=True)
