set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3w4; mkdir -p $o
WT_COMPACT=1 timeout -k 10 200 python tools/wave_times.py 1048576 c2 > $o/c2.log 2>&1 || exit $?
timeout -k 10 200 python tools/wave_times.py 1048576 c2 > $o/c2_full.log 2>&1 || exit $?
