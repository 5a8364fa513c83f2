# round 4, session 12: the GPU suite on the in-tree build (adds the one-request-per-lane class fill,
# flag 268435456, to the value-class and full-size routing tests), then that fill against the quad
# fill on C4, settings alternated in one process
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s12; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
AB_COMPACT=1 timeout -k 10 300 python tools/ab.py c4 "" "MXP_DEBUG_FLAGS=268435456" > $o/ab_c4_r1.log 2>&1 || exit $?
