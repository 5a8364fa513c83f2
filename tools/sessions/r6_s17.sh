# round 6, session 17: regex union walk over lookups bucketed by their first three bytes (A/B), list tests
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s17; mkdir -p $o
timeout -k 10 200 python -u tools/ab_rxp.py > $o/ab_rxp.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_lists.py tests/test_gpu_regex_nfa.py -m gpu -q --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log; [ $rc -ge 124 ] && exit $rc
exit 0
