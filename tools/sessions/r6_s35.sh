# round 6, session 35: pair Resolve (the selected rules from the evaluation's filed deferred pairs, the
# match bitmap never written): its tests, the resolver / group / dtp suites, then the end-to-end C2
# calls with it (MXP_RESOLVE_PAIRS=1) and without (0) alternated, then rocprofv3 of the calls
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1 GPU_MAX_HW_QUEUES=8
o=gpurun_out/r6s35; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_pair_resolve.py -m gpu -v -x --timeout 300 --timeout-method thread > $o/t0.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t0.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_resolver.py tests/test_gpu_group.py tests/test_gpu_dtp.py -m gpu -q -x --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in 1 0; do
    echo "pairs=$v" >> $o/ab.log
    MXP_RESOLVE_PAIRS=$v timeout -k 10 200 python -u tools/e2e_group_prof.py c2 5 2>&1 | grep ms_per_batch >> $o/ab.log || exit $?
  done
done
bash tools/prof_e2e.sh r6s35 c2 > $o/prof.log 2>&1 || exit $?
exit 0
