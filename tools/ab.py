"""A/B timing of engine settings (environment knobs read at engine creation: MXP_GPW,
MXP_DEBUG_FLAGS, ...) on one workload, alternated over repetitions in one process so box-to-box
variance cancels.  usage: ab.py c2|c4|c4p "MXP_GPW=4" "MXP_GPW=8" ..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from istio_amd import workloads as W  # noqa: E402
from istio_amd.engine import Engine  # noqa: E402

wl, settings = sys.argv[1], sys.argv[2:]
if wl == "c4":
    manifest, rules, batch = W.c4_workload(n_rules=10000, n_requests=1 << 20, seed=4)
elif wl == "c4p":  # C4 route rules matched on paths alone (no value classes)
    manifest, rules, batch = W.c4_workload(n_rules=10000, n_requests=1 << 20, seed=4, paths_only=True)
else:
    manifest, rules, batch = W.c2_workload(n_rules=10000, n_requests=1 << 20, seed=2)
Wd = (len(rules) + 31) // 32
dm = torch.empty((Wd, batch.n), dtype=torch.int32, device="cuda:0")
de = torch.empty_like(dm)
hits = torch.zeros(len(rules), dtype=torch.int64, device="cuda:0")
flags = torch.empty(batch.n, dtype=torch.uint8, device="cuda:0")
compact = bool(os.environ.get("AB_COMPACT"))  # the bench's error output (per-request flags)
loop = int(os.environ.get("AB_LOOP", "1"))  # evaluations back to back per timed interval (the bench's loop)


def ev(db, s):
    if compact:
        db.eval_compact(dm.data_ptr(), flags.data_ptr(), hits.data_ptr(), s.cuda_stream)
    else:
        db.eval_hits(dm.data_ptr(), de.data_ptr(), hits.data_ptr(), s.cuda_stream)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
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
        for _ in range(3):
            ev(db, s)
        ts = []
        for _ in range(15):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(loop):
                ev(db, s)
            b.record(s)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) / loop)
        res[st].append(float(np.median(ts)))
        db.free()
        del eng
for st, v in res.items():
    print("%s %-28s ms/eval %s  median %.3f" % (wl, st or "(default)", ["%.3f" % x for x in v], np.median(v)), flush=True)
