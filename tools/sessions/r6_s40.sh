# round 6, session 40: pair passes with packed chunk counts (rolled loop) and err_in loaded beside nsinfo: tests, e2e, rocprofv3
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1 GPU_MAX_HW_QUEUES=8
o=gpurun_out/r6s40; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_pair_resolve.py tests/test_gpu_resolver.py -m gpu -q -x --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  timeout -k 10 200 python -u tools/e2e_group_prof.py c2 5 2>&1 | grep ms_per_batch >> $o/e2e.log || exit $?
done
bash tools/prof_e2e.sh r6s40 c2 > $o/prof.log 2>&1 || exit $?
exit 0
