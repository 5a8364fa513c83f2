# round 5, session 7: the download / resolver / pack / list / quota GPU tests on the shader-copy
# downloads, batched resolve walk and split batch check; the C2 and C4 traces; pipelined Resolve;
# the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s7; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_download.py tests/test_gpu_resolver.py tests/test_batch_check.py \
  tests/test_gpu_pack.py tests/test_gpu_lists.py tests/test_gpu_memquota.py tests/test_gpu_bin.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/e2e_trace.py --workload c2 > $o/e2e_c2.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/e2e_trace.py --workload c4 > $o/e2e_c4.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/e2e_pipe.py --workload c2 --engines 3 --calls 8 > $o/pipe_c2.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/e2e_pipe.py --workload c4 --engines 2 --calls 4 > $o/pipe_c4.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --no-cpu-baseline > $o/bench.log 2>&1 || exit $?
