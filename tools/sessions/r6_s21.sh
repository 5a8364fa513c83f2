# round 6, session 21: the Resolve count pass reading four consecutive requests' words with one
# 16-byte load (mxp_resolve_count4v_kernel) against the strided kernel: resolver tests, then the
# end-to-end C2 call alternated (MXP_RESOLVE_VEC=1 / 0) and a kernel table of both.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1 GPU_MAX_HW_QUEUES=8
o=gpurun_out/r6s21; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_resolver.py tests/test_gpu_group.py -m gpu -q -x --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in 1 0; do
    echo "vec $v" >> $o/ab.log
    MXP_RESOLVE_VEC=$v timeout -k 10 200 python -u tools/e2e_group_prof.py c2 5 2>&1 | grep ms_per_batch >> $o/ab.log || exit $?
  done
done
for v in 1 0; do
  MXP_RESOLVE_VEC=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof$v -o e2e -- python3 -u tools/e2e_group_prof.py c2 3 > $o/prof$v.log 2>&1 || exit $?
done
exit 0
