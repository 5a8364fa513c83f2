# round 4, session 9: the GPU suite on the in-tree build (first-table direct postings carry their
# aliases, word-wise string copy, 2-D mark / gather grids), then same-box A/B: C2 r4s8a -> r4s8b
# (prefix keys inline), C4 / C2 r4s8b -> r4s9c (alias postings), C4 value-class fill tiles per
# workgroup 4 -> 8 / 2, and the packer's kernels under rocprof (interning ablations: no pool probe;
# loads and stores only)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s9; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4s8b.so ablib/libmxp_r4s9c.so > $o/ab_c4_alias.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_r4s8b.so ablib/libmxp_r4s9c.so > $o/ab_c2_alias.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_r4s8a.so ablib/libmxp_r4s8b.so > $o/ab_c2_inline.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4s8b.so ablib/libmxp_r4s9_t8.so > $o/ab_c4_t8.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4s8b.so ablib/libmxp_r4s9_t2.so > $o/ab_c4_t2.log 2>&1 || exit $?
for lib in ablib/libmxp_r4s8b.so ablib/libmxp_r4s9_nopool.so ablib/libmxp_r4s9_floor.so ablib/libmxp_r4s9c.so; do
    n=$(basename $lib .so)
    MXP_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/up_$n -o run -- python3 tools/upload_prof.py c2 4 > $o/up_$n.log 2>&1 || exit $?
done
MXP_LIB=ablib/libmxp_r4s9c.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/up4_r4s9c -o run -- python3 tools/upload_prof.py c4 4 > $o/up4_r4s9c.log 2>&1 || exit $?
