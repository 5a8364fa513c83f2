set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3s16; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_dtp.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_base.so ablib/libmxp_sort16.so > $o/ab_c4.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_base.so ablib/libmxp_sort16.so > $o/ab_c2.log 2>&1 || exit $?
MXP_LIB=ablib/libmxp_sort16.so bash tools/prof_session.sh r3s16/prof > $o/prof.log 2>&1 || exit $?
