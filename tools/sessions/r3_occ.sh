set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3o; mkdir -p $o
for wl in c2 c4; do
for lib in ablib/libmxp_v2.so ablib/libmxp_ix5.so ablib/libmxp_ix4.so ablib/libmxp_ix5.so ablib/libmxp_v2.so; do
  echo "== $lib" >> $o/ab_$wl.log
  AB_COMPACT=1 MXP_LIB=$lib timeout -k 10 200 python tools/ab.py $wl "" >> $o/ab_$wl.log 2>&1 || exit $?
done
done
