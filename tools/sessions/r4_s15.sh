# round 4, session 15: the GPU suite on the in-tree build (IPv4 /16 directory for CIDR lists), then
# the C3 CIDR block with and without it (r4s14a: binary search over the whole interval set),
# processes alternated
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s15; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
for lib in ablib/libmxp_r4s14a.so istio_amd/libmxp.so istio_amd/libmxp.so ablib/libmxp_r4s14a.so; do
    echo "== $lib" >> $o/ab_c3ip.log
    MXP_LIB=$lib timeout -k 10 200 python bench.py --workload c3-ip --no-cpu-baseline --steps 20 --warmup 5 >> $o/ab_c3ip.log 2>&1 || exit $?
done
