"""Fill-kernel store policy experiment (MXP_DEBUG_FLAGS 128 = non-temporal stores): C2 10k x 1M,
ms per evaluation from HIP events, both policies alternated."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from istio_amd import workloads as W  # noqa: E402
from istio_amd.engine import Engine  # noqa: E402

manifest, rules, batch = W.c2_workload(n_rules=10000, n_requests=1 << 20, seed=2)
res = {}
outs = {}
for flags in ["0", "128", "0", "128"]:
    os.environ["MXP_DEBUG_FLAGS"] = flags
    eng = Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    db = eng.upload(batch)
    Wd = (len(rules) + 31) // 32
    dm = torch.empty((Wd, batch.n), dtype=torch.int32, device="cuda:0")
    de = torch.empty_like(dm)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    eng.set_timing(True)
    for _ in range(3):
        db.eval(dm.data_ptr(), de.data_ptr(), s.cuda_stream)
    ts, kk = [], []
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        db.eval(dm.data_ptr(), de.data_ptr(), s.cuda_stream)
        b.record(s)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
        kk.append(eng.kernel_times())
    res.setdefault(flags, []).append((np.median(ts), np.median([k[0] for k in kk]), np.median([k[1] for k in kk])))
    outs[flags] = (dm.cpu().numpy().copy(), de.cpu().numpy().copy())
    db.free()
for f, v in res.items():
    print("flags", f, ["eval %.3f ms (fill+guard %.3f, index %.3f)" % x for x in v], flush=True)
print("identical outputs:", all(np.array_equal(a, b) for a, b in zip(outs["0"], outs["128"])))
