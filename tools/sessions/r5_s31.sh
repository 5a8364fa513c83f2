# round 5, session 31: ablation -- the guard-index kernel without its deferred-pair appends (ablib
# nopush; results invalid): what the appends cost the index kernel on C4 and C2.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s31; mkdir -p $o
sha1sum istio_amd/libmxp.so ablib/*.so > $o/libs.txt
for wl in c4 c2; do
  for v in base nopush; do
    if [ $v = base ]; then unset MXP_LIB; else export MXP_LIB=ablib/libmxp_nopush.so; fi
    timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $o/kt_${wl}_$v -o kt -- \
      python3 bench.py --no-cpu-baseline --no-c4 --no-c5 --no-c3 --fresh-steps 0 --e2e-reps 0 --steps 20 --warmup 3 --workload $wl > $o/kt_${wl}_$v.log 2>&1 || exit $?
  done
done
