# round 4, session 10: the GPU suite on the in-tree build (value-class fill group loop unrolled at
# compile time with a 64-bit deferred-pair merge; sort-kernel counters without same-word lanes and
# run-length hit counts; longest string from the scan kernels instead of a per-wave atomic; word-wise
# string copy), then same-box A/B r4s8b -> r4s10b (C4, C2), r4s10ns (sort kernel at HEAD) -> r4s10b
# (C4), and the packer's kernels under rocprof (C2, C4)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s10; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4s8b.so ablib/libmxp_r4s10b.so > $o/ab_c4.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4s10ns.so ablib/libmxp_r4s10b.so > $o/ab_c4_sort.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_r4s8b.so ablib/libmxp_r4s10b.so > $o/ab_c2.log 2>&1 || exit $?
for w in c2 c4; do
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/up_$w -o run -- python3 tools/upload_prof.py $w 4 > $o/up_$w.log 2>&1 || exit $?
done
