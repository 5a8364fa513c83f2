# round 5, session 2: resolver / bin / batch-check / list GPU tests (compact Resolve path, IP family
# split, inline string slots), end-to-end traces (pinned vs pageable, u16 vs u32) for C2 and C4, list
# A/B (IP split on/off in one process; string slots against the previous build, processes
# alternated), then the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s2; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_resolver.py tests/test_gpu_bin.py tests/test_batch_check.py tests/test_gpu_refs.py tests/test_gpu_lists.py -m gpu -q --timeout 200 --timeout-method thread > $o/t.log 2>&1
rc=$?; [ $rc -ge 2 ] && exit $rc  # (test failures: go on; a crash or time limit: stop)
timeout -k 10 200 python -u tools/e2e_trace.py --workload c2 > $o/e2e_c2.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/e2e_trace.py --workload c2 --pageable --u32 > $o/e2e_c2_pageable.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/e2e_trace.py --workload c4 > $o/e2e_c4.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/ab_lists.py c3-ip "MXP_LIST_IP_SPLIT=1" "MXP_LIST_IP_SPLIT=0" > $o/ab_c3ip_split.log 2>&1 || exit $?
for lib in istio_amd/libmxp.so ablib/libmxp_r5_prelists.so ablib/libmxp_r5_prelists.so istio_amd/libmxp.so; do
    MXP_LIB=$lib timeout -k 10 120 python -u tools/ab_lists.py c3-str "" >> $o/ab_c3str_slots.log 2>&1 || exit $?
done
timeout -k 10 500 python -u bench.py --no-cpu-baseline > $o/bench.log 2>&1 || exit $?
