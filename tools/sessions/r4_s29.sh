#!/bin/bash
# round 4, session 29: the bench's per-step timing events (and C5's fork / join) without the
# system-scope fence: default bench line twice each way, alternated (BENCH_FENCED_EVENTS=1: torch's
# default events), then the C5 two-stream and bench-step GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s29; mkdir -p $o
for k in 1 2; do
    BENCH_FENCED_EVENTS=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --fresh-steps 0 --e2e-reps 0 > $o/bench_fenced_$k.log 2>&1 || exit $?
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --fresh-steps 0 --e2e-reps 0 > $o/bench_nofence_$k.log 2>&1 || exit $?
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r4s29/bench_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f.split("/")[-1], "c2 %.4f" % d["ms_per_step"], "eval %.4f" % d["eval_ms"],
                  " ".join("%s %.4f" % (k, d[k]["ms_per_step"]) for k in ("c4", "c5") if isinstance(d.get(k), dict)))
PY
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -x -q --timeout 120 --timeout-method thread > $o/gpu_scale.log 2>&1 || { tail -30 $o/gpu_scale.log; exit 1; }
tail -2 $o/gpu_scale.log
