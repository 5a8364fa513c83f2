set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3sc; mkdir -p $o
MXP_LIB=ablib/libmxp_sc.so timeout -k 10 400 python -u -m pytest tests/test_gpu_dtp.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_t4.so ablib/libmxp_sc.so > $o/ab_c4.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_t4.so ablib/libmxp_sc.so > $o/ab_c2.log 2>&1 || exit $?
MXP_LIB=ablib/libmxp_sc.so bash tools/prof_session.sh r3sc/prof > $o/prof.log 2>&1 || exit $?
MXP_LIB=ablib/libmxp_sc.so bash tools/pmc_session.sh r3sc/pmc_c2 > $o/pmc_c2.log 2>&1 || exit $?
MXP_LIB=ablib/libmxp_sc.so bash tools/pmc_session.sh r3sc/pmc_c4 --workload c4 > $o/pmc_c4.log 2>&1 || exit $?
