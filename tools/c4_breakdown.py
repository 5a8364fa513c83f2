"""Where C4's evaluation time goes: the C4 requests against each rule class alone (prefix
startsWith, path regexps, header equality, header regexps), ms per evaluation (guard+VM / index)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from istio_amd import workloads as W  # noqa: E402
from istio_amd.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
manifest, rules, batch = W.c4_workload(n_rules=10000, n_requests=n, seed=4)
classes = {
    "all": rules,
    "startsWith": [r for r in rules if r.startswith("request.path.startsWith")],
    "path-regex": [r for r in rules if r.startswith('"^/')],
    "header-eq": [r for r in rules if r.startswith("request.headers")],
    "header-regex": [r for r in rules if r.startswith('"^v')],
}
only = os.environ.get("CLASSES")
for name, rs in classes.items():
    if only and name not in only.split(","):
        continue
    eng = Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rs)
    db = eng.upload(batch)
    Wd = (len(rs) + 31) // 32
    dm = torch.empty((Wd, batch.n), dtype=torch.int32, device="cuda:0")
    de = torch.empty_like(dm)
    hits = torch.zeros(len(rs), dtype=torch.int64, device="cuda:0")
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    eng.set_timing(True)
    for _ in range(2):
        db.eval(dm.data_ptr(), de.data_ptr(), s.cuda_stream)
    kk = []
    for _ in range(5):
        db.eval(dm.data_ptr(), de.data_ptr(), s.cuda_stream)
        kk.append(eng.kernel_times())
    db.eval_hits(dm.data_ptr(), de.data_ptr(), hits.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    tp = int(hits.sum().item()) / batch.n
    k = np.median(np.array(kk), axis=0)
    print("GPW=%s " % os.environ.get("MXP_GPW", "4") + "%-13s rules %5d  guard+VM %.3f ms  index %.3f ms  true pairs/request %.1f  info %s" % (
        name, len(rs), k[0], k[1] if len(k) > 1 else 0.0, tp, eng.ruleset_info()), flush=True)
    db.free()
