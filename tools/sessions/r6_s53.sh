# round 6, session 53: a narrow batch's column widen kernels queued after all column copies (one
# copy-to-kernel hand-off on the copy stream): narrow / pack / pair-Resolve / group tests, then the
# end-to-end C2 calls alternated with MXP_WIDEN_INTERLEAVE=1 (each widen behind its copy)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1 GPU_MAX_HW_QUEUES=8
o=gpurun_out/r6s53; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_pack.py tests/test_gpu_pair_resolve.py tests/test_gpu_group.py tests/test_gpu_async_upload.py -m gpu -q -x --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  echo "defer" >> $o/e2e.log
  timeout -k 10 200 python -u tools/e2e_group_prof.py c2 5 2>&1 | grep ms_per_batch >> $o/e2e.log || exit $?
  echo "interleave" >> $o/e2e.log
  MXP_WIDEN_INTERLEAVE=1 timeout -k 10 200 python -u tools/e2e_group_prof.py c2 5 2>&1 | grep ms_per_batch >> $o/e2e.log || exit $?
done
exit 0
