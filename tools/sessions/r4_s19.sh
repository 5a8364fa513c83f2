# round 4, session 19: the GPU suite on the in-tree build (the class fill skips the slots a group
# names no rule of), then same-box A/B r4s19base -> r4s19a on C4
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s19; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4s19base.so ablib/libmxp_r4s19a.so > $o/ab_c4.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4s19base.so ablib/libmxp_r4s19a.so > $o/ab_c4b.log 2>&1 || exit $?
