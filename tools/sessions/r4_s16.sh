# round 4, session 16: the GPU suite on the in-tree build (CIDR lookups: IPv4 parsed from registers,
# /16 directory; the C5 step's memquota batch on a second stream), then C3 CIDR in-tree vs r4s14a
# and C5 two streams vs --quota-serial, processes alternated
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s16; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
for lib in ablib/libmxp_r4s14a.so istio_amd/libmxp.so istio_amd/libmxp.so ablib/libmxp_r4s14a.so; do
    echo "== $lib" >> $o/ab_c3ip.log
    MXP_LIB=$lib timeout -k 10 200 python bench.py --workload c3-ip --no-cpu-baseline --steps 20 --warmup 5 >> $o/ab_c3ip.log 2>&1 || exit $?
done
for opt in "" "--quota-serial" "--quota-serial" ""; do
    echo "== c5 $opt" >> $o/ab_c5.log
    timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --e2e-reps 0 --fresh-steps 0 $opt >> $o/ab_c5.log 2>&1 || exit $?
done
