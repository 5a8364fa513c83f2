# round 4, session 11: the GPU suite on the in-tree build (string interning without scratch, class
# dictionary tiles with per-lane LDS counts and an insertion list; sort kernel and the fill's rolled
# group loop back at HEAD; the fill's 64-bit deferred-pair merge kept), then same-box A/B r4s8b ->
# r4s11a (C4: the merge alone; C2: no kernel change), the packer's kernels under rocprof (C2, C4)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s11; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4s8b.so ablib/libmxp_r4s11a.so > $o/ab_c4.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_r4s8b.so ablib/libmxp_r4s11a.so > $o/ab_c2.log 2>&1 || exit $?
for w in c2 c4; do
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/up_$w -o run -- python3 tools/upload_prof.py $w 4 > $o/up_$w.log 2>&1 || exit $?
done
