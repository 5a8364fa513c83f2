# round 6, session 22: the vector count pass with 8 vs 16 word rows in flight (MXP_RESOLVE_CW16)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1 GPU_MAX_HW_QUEUES=8
o=gpurun_out/r6s22; mkdir -p $o
for v in 0 1; do
  MXP_RESOLVE_CW16=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof$v -o e2e -- python3 -u tools/e2e_group_prof.py c2 3 > $o/prof$v.log 2>&1 || exit $?
done
exit 0
