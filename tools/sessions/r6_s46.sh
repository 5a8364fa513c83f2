# round 6, session 46: pair Resolve over ragged batch sizes (0, 1, 3, 5, 1000, 1025, 4097, 66001
# requests; one engine and a two-member group) against the bitmap Resolve
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s46; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_pair_resolve.py -m gpu -v -x --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log
exit $rc
