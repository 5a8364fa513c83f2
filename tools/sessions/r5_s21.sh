# round 5, session 21: why the unrolled value-class fill measured slower (s20): C4 SQ counters and
# kernel durations for the closing build (ablib r5base) and the unrolled one (in-tree).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s21; mkdir -p $o
sha1sum istio_amd/libmxp.so ablib/*.so > $o/libs.txt
for v in base new; do
  if [ $v = base ]; then export MXP_LIB=ablib/libmxp_r5base.so; else unset MXP_LIB; fi
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $o/kt_$v -o kt -- \
    python3 bench.py --no-cpu-baseline --no-c4 --no-c5 --no-c3 --fresh-steps 0 --e2e-reps 0 --steps 20 --warmup 3 --workload c4 > $o/kt_$v.log 2>&1 || exit $?
  bash tools/sq_session.sh r5s21/sq_$v --workload c4 > $o/sq_$v.log 2>&1 || exit $?
done
