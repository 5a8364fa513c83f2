# round 4, session 22: C2's VM passes ablated (every queued pair true: results invalid, an upper
# bound on what evaluating the continuation inline could save), settings alternated in one process
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s22; mkdir -p $o
MXP_LIB=ablib/libmxp_r4s22novm.so AB_COMPACT=1 timeout -k 10 300 python tools/ab.py c2 "" "MXP_DEBUG_FLAGS=16384" > $o/ab_c2_novm.log 2>&1 || exit $?
