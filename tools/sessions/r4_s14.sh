# round 4, session 14: the deferred-pair sort at 2 and 4 workgroups per tile (r4s13s2 / r4s13s4)
# against 1 (r4s13a), C4 and C2 same-box; the C4 index-wave timeline after the per-wave appends
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s14; mkdir -p $o
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4s13a.so ablib/libmxp_r4s13s2.so > $o/ab_c4_s2.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4s13a.so ablib/libmxp_r4s13s4.so > $o/ab_c4_s4.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_r4s13a.so ablib/libmxp_r4s13s2.so > $o/ab_c2_s2.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_r4s13a.so ablib/libmxp_r4s13s4.so > $o/ab_c2_s4.log 2>&1 || exit $?
MXP_LIB=ablib/libmxp_r4s13a.so WT_COMPACT=1 timeout -k 10 300 python tools/wave_times.py > $o/wave_times_c4.log 2>&1 || exit $?
