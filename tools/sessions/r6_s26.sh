# round 6, session 26: the u32 id check without the limit table (vectorised): narrow and batch-check
# tests, then the fresh-batch and end-to-end C2 loops (upload call host time)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1 GPU_MAX_HW_QUEUES=8
o=gpurun_out/r6s26; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_narrow.py tests/test_batch_check.py -m gpu -q -x --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 200 python -u tools/fresh_group_prof.py c2 10 narrow >> $o/ab.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/e2e_group_prof.py c2 5 >> $o/ab.log 2>&1 || exit $?
done
exit 0
