# round 6, session 45: mxp_dtp_sort_kernel's lanes take list entries 8 apart (distinct quads per
# atomic instruction): parity over the deferred pairs, then a same-box A/B against the previous
# build (abbase/libmxp_base.so) on C4 and C2, processes alternated
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s45; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_pair_resolve.py tests/test_gpu_group.py -m gpu -q -x --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log; [ $rc -ne 0 ] && exit $rc
AB_COMPACT=1 AB_LOOP=20 bash tools/ab_libs.sh c4 abbase/libmxp_base.so istio_amd/libmxp.so > $o/ab_c4.log 2>&1 || exit $?
AB_COMPACT=1 AB_LOOP=20 bash tools/ab_libs.sh c2 abbase/libmxp_base.so istio_amd/libmxp.so > $o/ab_c2.log 2>&1 || exit $?
exit 0
