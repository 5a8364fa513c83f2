set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3ck; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_gpu_heads.py tests/test_gpu_parity.py tests/test_gpu_dtp.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || exit $?
for lib in ablib/libmxp_vterr.so ablib/libmxp_ckey.so ablib/libmxp_vterr.so ablib/libmxp_ckey.so; do
  echo "== $lib" >> $o/steady_c2.log
  MXP_LIB=$lib timeout -k 10 200 python tools/steady.py c2 >> $o/steady_c2.log 2>&1 || exit $?
done
