set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3chp; mkdir -p $o
MXP_DTP_CHUNKS=2 AB_COMPACT=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/p2 -o run -- python3 tools/ab.py c2 "" > $o/p2.log 2>&1 || exit $?
