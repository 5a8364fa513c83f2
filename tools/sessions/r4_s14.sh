# round 4, session 14: the GPU suite on the in-tree build (occupancy bitmaps of the prefix /
# composite pair tables read before an entry pair), then bitmaps on vs off (MXP_DEBUG_FLAGS 4),
# settings alternated in one process, C4 and C2
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s14; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
AB_COMPACT=1 timeout -k 10 300 python tools/ab.py c4 "" "MXP_DEBUG_FLAGS=4" > $o/ab_c4_hbits.log 2>&1 || exit $?
AB_COMPACT=1 timeout -k 10 300 python tools/ab.py c2 "" "MXP_DEBUG_FLAGS=4" > $o/ab_c2_hbits.log 2>&1 || exit $?
