set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3dbg; mkdir -p $o
MXP_LIB=ablib/libmxp_lite.so timeout -k 10 200 python tools/dbg/vt_hits_check.py > $o/lite.log 2>&1 || exit $?
MXP_LIB=ablib/libmxp_vtrow.so timeout -k 10 200 python tools/dbg/vt_hits_check.py > $o/vtrow.log 2>&1 || exit $?
