# round 5, session 16: the packer's uploads as one gather kernel per group -- async-upload / pack /
# resolver tests, the fresh-batch timeline, the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s16; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib.sha1
timeout -k 10 600 python -u -m pytest tests/test_gpu_async_upload.py tests/test_gpu_pack.py tests/test_gpu_bin.py \
  tests/test_gpu_resolver.py tests/test_gpu_heads.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $o/fresh_c2 -o run -- \
  python3 tools/fresh_prof.py c2 8 > $o/fresh_c2.log 2>&1 || exit $?
python3 tools/copy_timeline.py $o/fresh_c2 4 > $o/timeline_c2.txt 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --no-cpu-baseline > $o/bench.log 2>&1 || exit $?
