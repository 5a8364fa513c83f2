# round 5, session 2: resolver / bin / batch-check GPU tests on the compact Resolve path, then the
# end-to-end trace (pinned vs pageable, u16 vs u32) for C2 and C4, then the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s2; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_resolver.py tests/test_gpu_bin.py tests/test_batch_check.py tests/test_gpu_refs.py -m gpu -x -q --timeout 200 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/e2e_trace.py --workload c2 > $o/e2e_c2.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/e2e_trace.py --workload c2 --pageable --u32 > $o/e2e_c2_pageable.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/e2e_trace.py --workload c4 > $o/e2e_c4.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --no-cpu-baseline > $o/bench.log 2>&1 || exit $?
