# round 6, session 39: the ids enqueued with the other outputs (guarded write, count-sized download), one synchronisation

set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1 GPU_MAX_HW_QUEUES=8
o=gpurun_out/r6s39; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_pair_resolve.py tests/test_gpu_resolver.py tests/test_gpu_group.py tests/test_gpu_download.py -m gpu -q -x --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  timeout -k 10 200 python -u tools/e2e_group_prof.py c2 5 2>&1 | grep ms_per_batch >> $o/e2e.log || exit $?
done
exit 0
