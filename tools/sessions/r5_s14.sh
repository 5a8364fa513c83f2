# round 5, session 14: no-wait uploads (MXP_UPLOAD_NO_WAIT) and the finish read-back on its own
# stream -- async-upload tests, the packing / bin / scale / resolver GPU tests, the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s14; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib.sha1
timeout -k 10 600 python -u -m pytest tests/test_gpu_async_upload.py tests/test_gpu_pack.py tests/test_gpu_bin.py \
  tests/test_gpu_scale.py tests/test_gpu_resolver.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --no-cpu-baseline > $o/bench.log 2>&1 || exit $?
