# round 5, session 4: the whole GPU suite (u16 regex-list parts), the resolver text diagnostic, the
# regex-list A/B (u16 sorted parts vs u32 in order), end-to-end traces, the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s4; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; [ $rc -ge 2 ] && exit $rc  # (test failures: go on; a crash or time limit: stop)
timeout -k 10 120 python -u tools/dbg/resolver_text.py bitmap > $o/dbg_resolver_bitmap.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/dbg/resolver_text.py compact > $o/dbg_resolver_compact.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_lists.py c3-regex "MXP_LIST_RX16=1" "MXP_LIST_RX16=0" > $o/ab_c3rx_16.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/e2e_trace.py --workload c2 > $o/e2e_c2.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/e2e_trace.py --workload c4 > $o/e2e_c4.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --no-cpu-baseline > $o/bench.log 2>&1 || exit $?
