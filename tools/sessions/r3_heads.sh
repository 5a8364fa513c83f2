# string heads A/B: r3 base build vs heads build (processes alternated), and MXP_HEADS=0/1 in one process
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3h; mkdir -p $o
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $o/parity.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_r3base.so ablib/libmxp_heads.so > $o/ab_c2.log 2>&1 || exit $?
AB_COMPACT=1 timeout -k 10 200 python tools/ab.py c2 MXP_HEADS=0 MXP_HEADS=1 > $o/ab_c2_flag.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r3base.so ablib/libmxp_heads.so > $o/ab_c4.log 2>&1 || exit $?
timeout -k 10 200 python tools/wave_times.py 1048576 c2 > $o/waves_c2.log 2>&1 || exit $?
