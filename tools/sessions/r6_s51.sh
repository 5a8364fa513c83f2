# round 6, session 51: the lite index kernel with the pair tables' occupancy bitmaps staged in LDS, folded on the host (OR of 2^F words) to 12 KB
# (mxp_index_dtp_lite_hb_kernel, 4 waves/SIMD): parity over the deferred pairs, which kernel C4 / C2
# take (rocprofv3), then the same build with staging off (MXP_DEBUG_FLAGS=16384) alternated in one process
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s51; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_pair_resolve.py tests/test_gpu_dtp.py tests/test_gpu_group.py -m gpu -q -x --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log; [ $rc -ne 0 ] && exit $rc
AB_COMPACT=1 AB_LOOP=5 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof_c4 -o run -- python3 tools/ab.py c4 "" > $o/prof_c4.log 2>&1 || exit $?
AB_COMPACT=1 AB_LOOP=5 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof_c2 -o run -- python3 tools/ab.py c2 "" > $o/prof_c2.log 2>&1 || exit $?
AB_COMPACT=1 AB_LOOP=20 timeout -k 10 300 python -u tools/ab.py c4 "" "MXP_DEBUG_FLAGS=16384" > $o/ab_c4.log 2>&1 || exit $?
AB_COMPACT=1 AB_LOOP=20 timeout -k 10 300 python -u tools/ab.py c2 "" "MXP_DEBUG_FLAGS=16384" > $o/ab_c2.log 2>&1 || exit $?
exit 0
