#!/bin/bash
# rocprofv3 kernel-trace summary of the default bench (no CPU baseline), into gpurun_out/$1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1
shift
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- python3 bench.py --no-cpu-baseline --e2e-reps 0 "$@" > "$out/bench.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
find "$out" -name "*kernel_stats.csv" -exec cp {} "$out/kernel_stats.csv" \;
cat "$out/kernel_stats.csv" 2>/dev/null | cut -d, -f1-4
exit $rc
