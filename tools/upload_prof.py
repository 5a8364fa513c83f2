"""Uploads of one synthetic batch, repeated (mxp_batch_upload: H2D copy + the device packer), for
rocprofv3 --kernel-trace --stats per packer kernel; prints the wall time per upload.
usage: upload_prof.py c2|c4 [reps]   (MXP_LIB picks the library: A/B of packer variants)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from istio_amd import workloads as W  # noqa: E402
from istio_amd.engine import Engine  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
if wl == "c4":
    manifest, rules, batch = W.c4_workload(n_rules=10000, n_requests=1 << 20, seed=4)
else:
    manifest, rules, batch = W.c2_workload(n_rules=10000, n_requests=1 << 20, seed=2)
eng = Engine(0)
eng.set_vocabulary(manifest)
eng.compile(rules)
ts = []
for i in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    db = eng.upload(batch)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
    db.free()
print("%s (%s) upload ms: %s" % (wl, os.environ.get("MXP_LIB", "in-tree"), " ".join("%.2f" % t for t in ts)))
