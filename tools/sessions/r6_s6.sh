# round 6, session 6: the default bench line (device group, narrow fresh / end-to-end batches,
# pipelined Resolve, regex-list prefix dispatch, packer scratch released after packing), twice.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s6; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib.sha1
timeout -k 10 300 python -u -m pytest tests/test_gpu_async_upload.py tests/test_gpu_narrow.py tests/test_gpu_bin.py tests/test_gpu_pack.py -m gpu -q --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 450 python -u bench.py --steps 20 --warmup 5 > $o/bench.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --wire wide --no-c3 --no-c5 > $o/bench_wide.log 2>&1 || exit $?
