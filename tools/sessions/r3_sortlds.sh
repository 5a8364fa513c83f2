set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3sl; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_dtp.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
for wl in c4 c2; do
  for cfg in "ablib/libmxp_sort16.so" "ablib/libmxp_lds.so" "ablib/libmxp_lds.so MXP_DTP_SORT_LDS=150" "ablib/libmxp_lds.so MXP_DTP_SORT_LDS=150" "ablib/libmxp_lds.so" "ablib/libmxp_sort16.so"; do
    set -- $cfg
    echo "== $cfg" >> $o/ab_$wl.log
    env AB_COMPACT=1 MXP_LIB=$1 ${2:-X_UNUSED=0} timeout -k 10 200 python tools/ab.py $wl "" >> $o/ab_$wl.log 2>&1 || exit $?
  done
done
bash tools/prof_session.sh r3sl/prof > $o/prof.log 2>&1 || exit $?
