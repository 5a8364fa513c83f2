# round 4, session 21: where C2's index wave goes now (wave timeline) and the probes-only ablation
# (MXP_DEBUG_FLAGS 1024: results invalid, an upper bound on the pair processing's share)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s21; mkdir -p $o
WT_COMPACT=1 timeout -k 10 300 python tools/wave_times.py 1048576 c2 > $o/wave_times_c2.log 2>&1 || exit $?
AB_COMPACT=1 timeout -k 10 300 python tools/ab.py c2 "" "MXP_DEBUG_FLAGS=1024" > $o/ab_c2_probes_only.log 2>&1 || exit $?
