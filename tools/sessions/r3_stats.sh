set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3st; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_dtp.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_sort.so ablib/libmxp_nostats.so > $o/ab_c2.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_sort.so ablib/libmxp_nostats.so > $o/ab_c4.log 2>&1 || exit $?
WT_COMPACT=1 timeout -k 10 200 python tools/wave_times.py 1048576 c2 > $o/waves_c2.log 2>&1 || exit $?
