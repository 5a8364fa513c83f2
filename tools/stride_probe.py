"""Do the batch's 2^k column strides cost anything?  The same rule set over a 2^20-request batch and
over its first 2^20 - 64 requests (columns then N - 64 apart, off every power of two), evaluated
alternately (20 back to back per timed interval); prints ms per evaluation scaled to 2^20 requests.
usage: stride_probe.py c2|c4"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from istio_amd import workloads as W  # noqa: E402
from istio_amd.engine import Engine  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
N = 1 << 20
mk = (lambda sh: W.c4_workload(n_rules=10000, n_requests=N, seed=4, shard=sh)) if wl == "c4" else \
     (lambda sh: W.c2_workload(n_rules=10000, n_requests=N, seed=2, shard=sh))
manifest, rules, full = mk(None)
_, _, cut = mk((0, N - 64))
eng = Engine(0)
eng.set_vocabulary(manifest)
eng.compile(rules)
R = len(rules)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
res = {}
for name, b in (("2^20", full), ("2^20-64", cut)):
    db = eng.upload(b)
    dm = torch.empty(((R + 31) // 32, b.n), dtype=torch.int32, device="cuda:0")
    fl = torch.empty(b.n, dtype=torch.uint8, device="cuda:0")
    hits = torch.zeros(R, dtype=torch.int64, device="cuda:0")
    res[name] = (db, dm, fl, hits, b.n, [])
for rep in range(6):
    for name, (db, dm, fl, hits, n, ts) in res.items():
        for _ in range(3):
            db.eval_compact(dm.data_ptr(), fl.data_ptr(), hits.data_ptr(), s.cuda_stream)
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(20):
            db.eval_compact(dm.data_ptr(), fl.data_ptr(), hits.data_ptr(), s.cuda_stream)
        e.record(s)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(e) / 20 * N / n)
for name, (_, _, _, _, n, ts) in res.items():
    print("%s %-8s n=%d ms/eval (per 2^20 requests) %s median %.4f" % (wl, name, n, ["%.4f" % t for t in ts], np.median(ts)),
          flush=True)
