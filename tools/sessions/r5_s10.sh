# round 5, session 10: the tiled Resolve walk -- resolver parity (tiled and per-lane), downloads;
# the C2 / C4 traces and their kernel tables.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s10; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib.sha1
timeout -k 10 500 python -u -m pytest tests/test_gpu_resolver.py tests/test_gpu_download.py tests/test_gpu_refs.py tests/test_gpu_errors.py tests/test_gpu_parity.py \
  -m gpu -x -v --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/e2e_trace.py --workload c2 --reps 2 > $o/e2e_c2.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/e2e_trace.py --workload c4 --reps 2 > $o/e2e_c4.log 2>&1 || exit $?
bash tools/prof_e2e.sh r5s10/prof c2 c4 > $o/prof.log 2>&1 || exit $?
