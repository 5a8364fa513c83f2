# round 4, session 8: same-box A/B r4s8base -> r4s8a (`.*$` tail-key postings, direct postings
# outside the pair queue, lite index kernel chosen over reachable templates), then the GPU suite
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s8; mkdir -p $o
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4s8base.so ablib/libmxp_r4s8a.so > $o/ab_c4.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_r4s8a.so ablib/libmxp_r4s8b.so > $o/ab_c4_inline.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_r4s8base.so ablib/libmxp_r4s8b.so > $o/ab_c2.log 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
WT_COMPACT=1 timeout -k 10 300 python tools/wave_times.py > $o/wave_times_c4.log 2>&1 || exit $?
# packer: the string interning pass with and without its batch table (ablation: timing only)
for lib in ablib/libmxp_r4s8a.so ablib/libmxp_r4s8_notable.so; do
    n=$(basename $lib .so)
    MXP_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/up_$n -o run -- python3 tools/upload_prof.py c2 6 > $o/up_$n.log 2>&1 || exit $?
done
# SQ counters of C4 (instruction mix, LDS conflicts per kernel) on the in-tree build
bash tools/sq_session.sh r4s8/sq_c4 --workload c4 > $o/sq_c4.log 2>&1 || exit $?
