set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3qr; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --workload c5-quota --no-cpu-baseline --steps 10 --warmup 2 > $o/bench.log 2>&1 || exit $?
find $o/prof -name "*kernel_stats.csv" -exec cp {} $o/kernel_stats.csv \;
