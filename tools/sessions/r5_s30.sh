# round 5, session 30: ablation -- the deferred-pair sort without its scattered 2-byte slot stores
# (ablib sortnostore; results invalid): how much of the sort's 68 us the stores are.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s30; mkdir -p $o
sha1sum istio_amd/libmxp.so ablib/*.so > $o/libs.txt
for v in base nostore; do
  if [ $v = base ]; then unset MXP_LIB; else export MXP_LIB=ablib/libmxp_sortnostore.so; fi
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $o/kt_$v -o kt -- \
    python3 bench.py --no-cpu-baseline --no-c4 --no-c5 --no-c3 --fresh-steps 0 --e2e-reps 0 --steps 20 --warmup 3 --workload c4 > $o/kt_$v.log 2>&1 || exit $?
done
