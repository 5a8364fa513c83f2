# round 6, session 5: the whole GPU suite (no -x: every failure listed), then the default bench line
# (device group, narrow fresh / end-to-end batches, pipelined Resolve, regex-list prefix dispatch).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s5; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib.sha1
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "suite rc=$rc" >> $o/t.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 450 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $o/bench.log 2>&1 || exit $?
