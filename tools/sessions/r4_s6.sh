# round 4, session 6: same-box A/B first (r4b -> r4c: literal-key regexp postings; r4h -> r4f / r4g:
# the immediate-offset vtfill group loop unrolled by four, 3 waves/SIMD / bounded to 4 with spills),
# then the GPU suite on the in-tree build (two-level class dictionary, word-wise interning), rocprof
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s6; mkdir -p $o
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4b.so ablib/libmxp_r4c.so > $o/ab_c4_litkeys.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4h.so ablib/libmxp_r4f.so > $o/ab_c4_unroll.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4h.so ablib/libmxp_r4g.so > $o/ab_c4_unroll_w4.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_base.so ablib/libmxp_r4f.so > $o/ab_c2.log 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
bash tools/prof_session.sh r4s6/prof --no-c3 > $o/prof.log 2>&1 || exit $?
