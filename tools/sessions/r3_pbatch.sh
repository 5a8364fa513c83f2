set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3pb; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_heads.py tests/test_gpu_parity.py tests/test_gpu_dtp.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_base.so ablib/libmxp_pb.so > $o/ab_c2.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_base.so ablib/libmxp_pb.so > $o/ab_c4.log 2>&1 || exit $?
