set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3l; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_dtp.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_heads.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/steady.py c2 MXP_DEBUG_FLAGS=8388608 "" > $o/steady_c2.log 2>&1 || exit $?
timeout -k 10 300 python tools/steady.py c4 MXP_DEBUG_FLAGS=8388608 "" > $o/steady_c4.log 2>&1 || exit $?
