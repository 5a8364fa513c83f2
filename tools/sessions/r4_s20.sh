# round 4, session 20: the GPU suite on HEAD plus the recycled-blocks test (uploads into a freed
# batch's blocks, evaluations still in flight, against a fresh engine)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s20; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
