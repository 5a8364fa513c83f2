# round 4, session 5: literal-key regexp rules as direct / exact postings (no VM pass), wide NFA
# walk, list NFA kernels, word-wise interning, two-level class dictionary at upload; GPU suite,
# same-box A/B (r4b = vtfill imm, r4c = + literal keys), rocprof stats of the bench
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s5; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4b.so ablib/libmxp_r4c.so > $o/ab_c4.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_base.so ablib/libmxp_r4c.so > $o/ab_c2.log 2>&1 || exit $?
bash tools/prof_session.sh r4s5/prof --no-c3 > $o/prof.log 2>&1 || exit $?
