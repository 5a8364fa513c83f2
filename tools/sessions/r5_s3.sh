# round 5, session 3: the whole GPU suite (compact Resolve with device first errors, recycled last
# batches, list register paths), end-to-end traces with pinned outputs, list A/B per knob (one
# process), the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s3; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; [ $rc -ge 2 ] && exit $rc  # (test failures: go on; a crash or time limit: stop)
timeout -k 10 200 python -u tools/e2e_trace.py --workload c2 > $o/e2e_c2.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/e2e_trace.py --workload c4 > $o/e2e_c4.log 2>&1 || exit $?
timeout -k 10 150 python -u tools/ab_lists.py c3-ip "MXP_LIST_OPT=255" "MXP_LIST_OPT=0" "MXP_LIST_OPT=1" "MXP_LIST_OPT=2" > $o/ab_c3ip_opt.log 2>&1 || exit $?
timeout -k 10 150 python -u tools/ab_lists.py c3-str "MXP_LIST_OPT=255" "MXP_LIST_OPT=0" > $o/ab_c3str_opt.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --no-cpu-baseline > $o/bench.log 2>&1 || exit $?
