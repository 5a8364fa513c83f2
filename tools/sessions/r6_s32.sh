# round 6, session 32: narrow device pack against the host pack (new parity test)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s32; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_pack.py -m gpu -q -x --timeout 300 --timeout-method thread > $o/t.log 2>&1
echo "tests rc=$?" >> $o/t.log
exit 0
