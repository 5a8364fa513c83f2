# round 6, session 29: four members on device 0 with each member's host loops capped to its share of
# the threads (par.h tl_thread_cap): the fresh-batch upload call's host time; group tests
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s29; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_narrow.py -m gpu -q -x --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log; [ $rc -ne 0 ] && exit $rc
MXP_BENCH_WATCHDOG=150 timeout -k 10 700 python -u bench.py --devices 0,0,0,0 --steps 5 --warmup 2 --no-cpu-baseline --no-c3 > $o/bench4.log 2> $o/bench4.err
echo "rc=$?" >> $o/bench4.err
exit 0
