set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3rep; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_gpu_vt.py tests/test_gpu_dtp.py tests/test_gpu_scale.py -q --timeout 300 --timeout-method thread > $o/tests1.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -q --timeout 300 --timeout-method thread > $o/tests2.log 2>&1
MXP_LIB=ablib/libmxp_lite.so timeout -k 10 900 python -u -m pytest tests/test_gpu_vt.py tests/test_gpu_dtp.py tests/test_gpu_scale.py -q --timeout 300 --timeout-method thread > $o/tests3.log 2>&1
exit 0
