# round 6, session 16: regex lists pick the union when it fits one part (auto), the list tests, the
# full GPU suite, then the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s16; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib.sha1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 450 python -u bench.py --steps 20 --warmup 5 > $o/bench.log 2>&1 || exit $?
exit 0
