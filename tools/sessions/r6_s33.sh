# round 6, session 33: the two-call Resolve (submit / finish, the next upload between them): group and
# resolver tests, then the pipelined end-to-end C2 loop with it (BENCH_PIPE_SUBMIT=1) and without (0),
# alternated
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1 GPU_MAX_HW_QUEUES=8
o=gpurun_out/r6s33; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_resolver.py -m gpu -q -x --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in 1 0; do
    echo "submit=$v" >> $o/ab.log
    BENCH_PIPE_SUBMIT=$v timeout -k 10 200 python -u tools/e2e_group_prof.py c2 5 2>&1 | grep ms_per_batch >> $o/ab.log || exit $?
  done
done
exit 0
