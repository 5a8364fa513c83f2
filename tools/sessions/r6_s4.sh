# round 6, session 4: the group / list / upload / narrow-batch GPU tests (regex-list literal-prefix
# dispatch, narrow uploads, Resolve over uploaded batches), the whole GPU suite, then the default
# bench line through the group.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s4; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib.sha1
timeout -k 10 300 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_lists.py tests/test_gpu_async_upload.py \
  tests/test_gpu_narrow.py -m gpu -q --timeout 300 --timeout-method thread > $o/t1.log 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 450 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $o/bench.log 2>&1 || exit $?
