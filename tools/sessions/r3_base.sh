# r3 baseline at HEAD: GPU tests, smoke, default bench, rocprof of the default bench
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3b; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $o/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --no-cpu-baseline --e2e-reps 0 > $o/bench_prof.log 2>&1 || exit $?
find $o/prof -name "*kernel_stats.csv" -exec cp {} $o/kernel_stats.csv \;
