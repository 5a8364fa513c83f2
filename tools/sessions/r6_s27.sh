# round 6, session 27: host phases of the narrow upload call (MXP_TRACE=1 host marks)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1 GPU_MAX_HW_QUEUES=8
o=gpurun_out/r6s27; mkdir -p $o
MXP_TRACE=1 timeout -k 10 200 python -u tools/fresh_group_prof.py c2 4 narrow > $o/trace.log 2>&1 || exit $?
exit 0
