# round 4, session 1: GPU suite at HEAD (ADVICE fixes + the deep-continuation test), then the
# contiguous-entry sort (r3_sortc.patch) against the base build, same box, builds alternated
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r4s1; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_base.so ablib/libmxp_sc.so > $o/ab_c4.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_base.so ablib/libmxp_sc.so > $o/ab_c2.log 2>&1 || exit $?
