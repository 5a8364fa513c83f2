# round 6, session 52: HIP API + kernel trace of the end-to-end C2 calls on the final build (single and pipelined)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1 GPU_MAX_HW_QUEUES=8
o=gpurun_out/r6s52; mkdir -p $o
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $o/prof -o e2e -- python3 -u tools/e2e_group_prof.py c2 3 > $o/prof.log 2>&1 || exit $?
exit 0
