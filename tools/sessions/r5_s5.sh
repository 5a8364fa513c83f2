# round 5, session 5: the whole GPU suite (bitmap Resolve collects its records again; stash; batched
# downloads; multi-stream D2H; column copies on a copy stream), end-to-end traces, the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s5; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; [ $rc -ge 2 ] && exit $rc  # (test failures: go on; a crash or time limit: stop)
timeout -k 10 200 python -u tools/e2e_trace.py --workload c2 > $o/e2e_c2.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/e2e_trace.py --workload c4 > $o/e2e_c4.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --no-cpu-baseline > $o/bench.log 2>&1 || exit $?
