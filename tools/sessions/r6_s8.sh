# round 6, session 8: regex dispatch with blocks up to 1 KB (no union part left on C3) and the
# tail classes loaded ahead of the walk; the group tests after the quota-download sync fix; bench.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s8; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib.sha1
timeout -k 10 200 python -u tools/ab_rxp.py > $o/ab_rxp.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_lists.py tests/test_gpu_regex_nfa.py tests/test_gpu_scale.py::test_c3_full_regex_union -m gpu -q --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log; [ $rc -ge 124 ] && exit $rc
# (then, with the group's non-blocking member streams and the async finish-path copies: the
# group / stream / pack tests and the default bench line)
timeout -k 10 400 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_async_upload.py tests/test_gpu_narrow.py tests/test_gpu_bin.py tests/test_gpu_pack.py tests/test_gpu_scale.py::test_c5_group_step -m gpu -q --timeout 300 --timeout-method thread > $o/t2.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t2.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 450 python -u bench.py --steps 20 --warmup 5 > $o/bench.log 2>&1 || exit $?
exit 0
