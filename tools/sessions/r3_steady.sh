set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3sd; mkdir -p $o
for lib in ablib/libmxp_fold.so ablib/libmxp_v9.so ablib/libmxp_fold.so ablib/libmxp_v9.so; do
  echo "== $lib" >> $o/steady_c2.log
  MXP_LIB=$lib timeout -k 10 200 python tools/steady.py c2 >> $o/steady_c2.log 2>&1 || exit $?
done
