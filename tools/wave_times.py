"""Index-kernel wave timeline on C4 (MXP_WAVE_TIMES hook): is the kernel's duration the waves' work
spread over the chip, or a tail of slow waves?  Prints the wave-duration distribution, the kernel span
and the number of waves in flight over time (per XCC)."""
import os
import sys

os.environ["MXP_WAVE_TIMES"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from istio_amd import workloads as W  # noqa: E402
from istio_amd.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
kind = sys.argv[2] if len(sys.argv) > 2 else "c4"
if kind == "c4":
    manifest, rules, batch = W.c4_workload(n_rules=10000, n_requests=n, seed=4)
else:
    manifest, rules, batch = W.c2_workload(n_rules=10000, n_requests=n, seed=2)
    rules = W.c2_rules(10000, seed=2)[0]
eng = Engine(0)
eng.set_vocabulary(manifest)
eng.compile(rules)
db = eng.upload(batch)
Wd = (len(rules) + 31) // 32
dm = torch.empty((Wd, batch.n), dtype=torch.int32, device="cuda:0")
de = torch.empty_like(dm)
compact = bool(os.environ.get("WT_COMPACT"))  # the bench's evaluation: compact errors, hit counters
hits = torch.zeros(len(rules), dtype=torch.int64, device="cuda:0")
flags = torch.zeros(batch.n, dtype=torch.uint8, device="cuda:0")


def one():
    if compact:
        db.eval_compact(dm.data_ptr(), flags.data_ptr(), hits.data_ptr(), 0)
    else:
        db.eval(dm.data_ptr(), de.data_ptr(), 0)


eng.set_timing(True)
for _ in range(3):
    one()
torch.cuda.synchronize()
if os.environ.get("WT_IDLE"):  # the last evaluation after an idle GPU (no fill write-back draining)
    import time
    time.sleep(0.05)
    one()
    torch.cuda.synchronize()
print("mxp_kernel_times of the last evaluation (ms):", eng.kernel_times(3))
t = eng.wave_times((n + 63) // 64).astype(np.int64)
start, end, xcc = t[:, 0], t[:, 1], t[:, 2] & 255
passes, runs, pairs = (t[:, 2] >> 8) & 0xFFFF, (t[:, 2] >> 24) & 0xFFFF, t[:, 2] >> 40
vm_us = t[:, 6] / 100.0
marks = t[:, 3:8].copy()
marks[:, 3] = 0  # (word 6 holds the run_pairs time)
dur = (end - start) / 100.0  # us
t0 = start.min()
print("%s: %d waves, kernel span %.1f us (first start -> last end)" % (kind, len(t), (end.max() - t0) / 100.0))
print("wave duration us: p50 %.1f p90 %.1f p99 %.1f max %.1f mean %.1f" % (
    np.percentile(dur, 50), np.percentile(dur, 90), np.percentile(dur, 99), dur.max(), dur.mean()))
for x in sorted(set(xcc.tolist())):
    m = xcc == x
    print("  XCC %d: %d waves, span %.1f us, mean %.1f us" % (x, m.sum(), (end[m].max() - start[m].min()) / 100.0,
                                                               dur[m].mean()))
edges = np.linspace(0, end.max() - t0, 21)
for a, b in zip(edges[:-1], edges[1:]):
    live = ((start - t0) < b) & ((end - t0) > a)
    print("  %7.1f-%7.1f us: %5d waves in flight, %5d started" % (a / 100, b / 100, live.sum(),
                                                                  (((start - t0) >= a) & ((start - t0) < b)).sum()))
slow = np.argsort(-dur)[:8]
print("slowest waves (index, us, start offset us):", [(int(i), round(float(dur[i]), 1), round(float((start[i] - t0) / 100), 1)) for i in slow])
# phases: start -> slot 0 -> slot 1 -> ... -> drain (per wave, us; 0 marks = slot not reached)
prev = start.copy()
first = (start - t0) < 200  # waves started in the kernel's first 2 us (the first round)
for k in range(5):
    m = marks[:, k]
    have = m > 0
    if not have.any():
        continue
    d = (m[have] - prev[have]) / 100.0
    f = first[have]
    print("phase %s: %d waves, p50 %.1f mean %.1f us; first round p50 %.1f, later p50 %.1f" % (
        "drain" if k == 4 else "slot %d" % k, have.sum(), np.percentile(d, 50), d.mean(),
        np.percentile(d[f], 50) if f.any() else 0.0, np.percentile(d[~f], 50) if (~f).any() else 0.0))
    prev = np.where(have, m, prev)
print("per wave: run_pairs time p50 %.1f mean %.1f us (%.0f%% of the wave); run_pairs calls %.1f, VM passes %.1f, pairs %.1f" % (
    np.percentile(vm_us, 50), vm_us.mean(), 100.0 * vm_us.sum() / max(dur.sum(), 1e-9), runs.mean(), passes.mean(), pairs.mean()))
