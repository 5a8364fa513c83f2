# round 6, session 47: a group larger than its batch (members with 0 or 1 requests): evaluation,
# counters and Resolve against one engine
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s47; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py -k few_or_no -m gpu -v -x --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/t.log
exit $rc
