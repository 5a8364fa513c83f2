# round 4, session 18: the GPU suite on the in-tree build (freed batches' device blocks recycled by
# later uploads instead of hipFree), then the fresh-batch loop with and without it (r4s18base)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s18; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
for w in c2 c4; do
    for lib in ablib/libmxp_r4s18base.so istio_amd/libmxp.so istio_amd/libmxp.so ablib/libmxp_r4s18base.so; do
        echo "== $w $lib" >> $o/ab_fresh.log
        MXP_LIB=$lib timeout -k 10 200 python tools/fresh_prof.py $w 10 >> $o/ab_fresh.log 2>&1 || exit $?
    done
done
