# round 6, session 42: the full bench line's pipelined C2 end-to-end period (2.41 ms) against the C2
# block alone (1.74 ms, r6_s41): which other workloads' inputs in the process slow it
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s42; mkdir -p $o
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/bench_all.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c3 > $o/bench_noc3.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c4 --no-c5 > $o/bench_noc4.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c3 --no-c4 --no-c5 > $o/bench_c2.log 2>&1 || exit $?
exit 0
