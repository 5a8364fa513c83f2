# round 5, session 32: ablation -- the index kernel's deferred-pair appends through lane-private
# slots (no same-address LDS atomic per pair; ablib lanepush, results invalid) against the in-tree
# build and no appends at all (ablib nopush): is the append cost the atomic or the stores?
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s32; mkdir -p $o
sha1sum istio_amd/libmxp.so ablib/*.so > $o/libs.txt
for v in base lanepush nopush; do
  if [ $v = base ]; then unset MXP_LIB; else export MXP_LIB=ablib/libmxp_$v.so; fi
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $o/kt_c4_$v -o kt -- \
    python3 bench.py --no-cpu-baseline --no-c4 --no-c5 --no-c3 --fresh-steps 0 --e2e-reps 0 --steps 20 --warmup 3 --workload c4 > $o/kt_c4_$v.log 2>&1 || exit $?
done
