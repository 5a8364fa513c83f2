# round 6, session 9: narrow uploads without the host widening (checks on the u32 arrays, the v1
# view made on demand), memquota replays forked at the last reduction; tests then the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s9; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib.sha1
timeout -k 10 500 python -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_group.py tests/test_batch_check.py tests/test_gpu_async_upload.py tests/test_gpu_pack.py tests/test_gpu_resolver.py tests/test_gpu_scale.py::test_c5_group_step tests/test_gpu_regex_nfa.py -m gpu -q --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 450 python -u bench.py --steps 20 --warmup 5 > $o/bench.log 2>&1 || exit $?
exit 0
