# round 6, session 44: deferred-pair request chunks (MXP_DTP_CHUNKS: chunk c's index and sort on a side
# stream beside chunk c - 1's fill) re-measured on the round-6 kernels (negative at r3), C4 and C2
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s44; mkdir -p $o
AB_COMPACT=1 AB_LOOP=20 timeout -k 10 300 python -u tools/ab.py c4 "" "MXP_DTP_CHUNKS=2" "MXP_DTP_CHUNKS=4" > $o/ab_c4.log 2>&1 || exit $?
AB_COMPACT=1 AB_LOOP=20 timeout -k 10 300 python -u tools/ab.py c2 "" "MXP_DTP_CHUNKS=2" "MXP_DTP_CHUNKS=4" > $o/ab_c2.log 2>&1 || exit $?
exit 0
