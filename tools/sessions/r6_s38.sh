# round 6, session 38: the resolver's device tables kept between calls and the compact Resolve's two
# counters downloaded into pinned memory together: pair / resolver / group tests, end-to-end C2 calls
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1 GPU_MAX_HW_QUEUES=8
o=gpurun_out/r6s38; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_pair_resolve.py tests/test_gpu_resolver.py tests/test_gpu_group.py -m gpu -q -x --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  timeout -k 10 200 python -u tools/e2e_group_prof.py c2 5 2>&1 | grep ms_per_batch >> $o/e2e.log || exit $?
done
exit 0
