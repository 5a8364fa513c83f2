# round 6, session 36: pair Resolve with the chunk counts prefetched (8 at a time): tests, end-to-end A/B, rocprofv3


set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1 GPU_MAX_HW_QUEUES=8
o=gpurun_out/r6s36; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_pair_resolve.py -m gpu -v -x --timeout 300 --timeout-method thread > $o/t0.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t0.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_resolver.py -m gpu -q -x --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in 1 0; do
    echo "pairs=$v" >> $o/ab.log
    MXP_RESOLVE_PAIRS=$v timeout -k 10 200 python -u tools/e2e_group_prof.py c2 5 2>&1 | grep ms_per_batch >> $o/ab.log || exit $?
  done
done
bash tools/prof_e2e.sh r6s36 c2 > $o/prof.log 2>&1 || exit $?
exit 0
