set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3ch; mkdir -p $o
MXP_DTP_CHUNKS=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_dtp.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
AB_COMPACT=1 timeout -k 10 300 python tools/ab.py c2 MXP_DTP_CHUNKS=1 MXP_DTP_CHUNKS=2 MXP_DTP_CHUNKS=4 MXP_DTP_CHUNKS=8 > $o/ab_c2.log 2>&1 || exit $?
AB_COMPACT=1 timeout -k 10 300 python tools/ab.py c4 MXP_DTP_CHUNKS=1 MXP_DTP_CHUNKS=2 MXP_DTP_CHUNKS=4 MXP_DTP_CHUNKS=8 > $o/ab_c4.log 2>&1 || exit $?
