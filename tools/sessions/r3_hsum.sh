set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3hs; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_gpu_dtp.py tests/test_gpu_scale.py tests/test_gpu_vt.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || exit $?
for wl in c2 c4; do
for lib in ablib/libmxp_ckey.so ablib/libmxp_hsum.so ablib/libmxp_ckey.so ablib/libmxp_hsum.so; do
  echo "== $lib" >> $o/steady_$wl.log
  MXP_LIB=$lib timeout -k 10 200 python tools/steady.py $wl >> $o/steady_$wl.log 2>&1 || exit $?
done
done
