#!/bin/bash
# round 4, session 30: C5's two streams at different priorities (evaluation stream high, memquota
# stream default; and the reverse), alternated, C5 block alone
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s30; mkdir -p $o
a="--workload c5 --no-c4 --no-c5 --no-c3 --no-cpu-baseline --fresh-steps 0 --e2e-reps 0 --steps 50"
for k in 1 2; do
    timeout -k 10 300 python -u bench.py $a > $o/c5_default_$k.log 2>&1 || exit $?
    BENCH_STREAM_PRIO=-1 timeout -k 10 300 python -u bench.py $a > $o/c5_evalhigh_$k.log 2>&1 || exit $?
    BENCH_QSTREAM_PRIO=-1 timeout -k 10 300 python -u bench.py $a > $o/c5_quotahigh_$k.log 2>&1 || exit $?
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r4s30/c5_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f.split("/")[-1], "ms/step %.4f" % d["ms_per_step"], "eval %.4f" % d["eval_ms"])
PY
