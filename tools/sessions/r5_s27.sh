# round 5, session 27: the slow value-class fill's workgroups scanning 16 fast-grid blocks' marks in
# parallel (in-tree, with the next-tile prefetch and the 4-request lookup) against the committed
# split fill (ablib split): parity, C4 steady state alternated, kernel durations.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s27; mkdir -p $o
sha1sum istio_amd/libmxp.so ablib/*.so > $o/libs.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_vt.py tests/test_gpu_dtp.py -m gpu -x -v \
  --timeout 200 --timeout-method thread > $o/t.log 2>&1 || exit $?
for k in 1 2; do
  for lib in ablib/libmxp_split.so ""; do
    echo "lib ${lib:-in-tree}" >> $o/ab_c4.log
    MXP_LIB=$lib timeout -k 10 200 python -u tools/steady.py c4 "" >> $o/ab_c4.log 2>&1 || exit $?
  done
done
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $o/kt_new -o kt -- \
  python3 bench.py --no-cpu-baseline --no-c4 --no-c5 --no-c3 --fresh-steps 0 --e2e-reps 0 --steps 20 --warmup 3 --workload c4 > $o/kt_new.log 2>&1 || exit $?
