# round 4, session 13: the GPU suite on the in-tree build (deferred-pair appends with one LDS atomic
# per wave instead of one per lane; the sort kernel's split constant at 1), then same-box A/B
# r4s12a -> r4s13a (the appends) on C4 and C2, the sort at 2 and 4 workgroups per tile (r4s13s2 /
# r4s13s4) against 1, and the C4 index-wave timeline
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s13; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4s12a.so ablib/libmxp_r4s13a.so > $o/ab_c4.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_r4s12a.so ablib/libmxp_r4s13a.so > $o/ab_c2.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4s13a.so ablib/libmxp_r4s13s2.so > $o/ab_c4_s2.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4s13a.so ablib/libmxp_r4s13s4.so > $o/ab_c4_s4.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_r4s13a.so ablib/libmxp_r4s13s2.so > $o/ab_c2_s2.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_r4s13a.so ablib/libmxp_r4s13s4.so > $o/ab_c2_s4.log 2>&1 || exit $?
MXP_LIB=ablib/libmxp_r4s13a.so WT_COMPACT=1 timeout -k 10 300 python tools/wave_times.py > $o/wave_times_c4.log 2>&1 || exit $?
