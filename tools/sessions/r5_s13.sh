# round 5, session 13: asynchronous device packing (upload returns after the copies; the first
# evaluation finishes the batch) -- the whole GPU suite, the C2 trace, the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s13; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib.sha1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/e2e_trace.py --workload c2 --reps 3 > $o/e2e_c2.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --no-cpu-baseline > $o/bench.log 2>&1 || exit $?
