# round 5, session 11: deferred error records -- error / resolver / parity / lists / refs GPU tests; C2 and C4 traces.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s11; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib.sha1
timeout -k 10 600 python -u -m pytest tests/test_gpu_errors.py tests/test_gpu_resolver.py tests/test_gpu_parity.py \
  tests/test_gpu_lists.py tests/test_gpu_refs.py tests/test_gpu_download.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/e2e_trace.py --workload c2 --reps 3 > $o/e2e_c2.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/e2e_trace.py --workload c4 --reps 2 > $o/e2e_c4.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/e2e_pipe.py --workload c2 --engines 3 --calls 8 > $o/pipe_c2.log 2>&1 || exit $?
