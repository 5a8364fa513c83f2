set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3w3; mkdir -p $o
timeout -k 10 200 python tools/wave_times.py 1048576 c2 > $o/c2.log 2>&1 || exit $?
timeout -k 10 200 python tools/wave_times.py 1048576 c4 > $o/c4.log 2>&1 || exit $?
