"""C4 at 1M: three compact evaluations with hit counters, then the per-rule bit counts of the match
bitmap; prints the rules whose counters disagree (debugging aid; MXP_LIB selects the build)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from istio_amd import workloads as W  # noqa: E402
from istio_amd.engine import Engine  # noqa: E402

manifest, rules, batch = W.c4_workload(n_rules=10_000, n_requests=1 << 20, seed=4)
R, N = len(rules), batch.n
eng = Engine(0)
eng.set_vocabulary(manifest)
eng.compile(rules)
db = eng.upload(batch)
Wd = (R + 31) // 32
dm = torch.zeros((Wd, N), dtype=torch.int32, device="cuda:0")
req_err = torch.zeros(N, dtype=torch.uint8, device="cuda:0")
hits = torch.zeros(R, dtype=torch.int64, device="cuda:0")
for _ in range(3):
    db.eval_compact(dm.data_ptr(), req_err.data_ptr(), hits.data_ptr(), 0)
torch.cuda.synchronize()
cnt = torch.zeros((Wd, 32), dtype=torch.int64, device="cuda:0")
for b in range(32):
    cnt[:, b] = ((dm >> b) & 1).sum(dim=1)
c = cnt.reshape(-1)[:R].cpu().numpy()
h = hits.cpu().numpy()
bad = np.nonzero(h != 3 * c)[0]
print("rules with bad counters:", len(bad))
for r in bad[:10]:
    print(r, rules[r][:70], "hits", h[r], "3*bits", 3 * c[r])
