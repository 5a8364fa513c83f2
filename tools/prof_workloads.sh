#!/bin/bash
# rocprofv3 kernel-trace summaries, one process per bench workload (C2, C4, C5, C3 ip / str / regex),
# so every kernel's average duration belongs to one workload: gpurun_out/$1/kernel_stats_<w>.csv.
# Steps only (no CPU baseline, no fresh-batch or end-to-end blocks): the upload kernels run once.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1
shift
mkdir -p "$out"
for w in c2 c4 c5 c3-ip c3-str c3-regex; do
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$w" -o run -- \
        python3 bench.py --workload $w --no-cpu-baseline --no-c4 --no-c5 --no-c3 --fresh-steps 0 --e2e-reps 0 "$@" \
        > "$out/bench_$w.log" 2>&1
    rc=$?
    echo "rocprof $w rc=$rc"
    [ $rc -ne 0 ] && exit $rc
    find "$out/$w" -name "*kernel_stats.csv" -exec cp {} "$out/kernel_stats_$w.csv" \;
done
exit 0
