# round 6, session 11: the fresh C2 loop with 4 / 8 / 16 hardware queues per process (the copy
# stream and the packer stream shared a queue at 4: copies of batch k + 1 waited for packer k).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s11; mkdir -p $o
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u tools/fresh_group_prof.py c2 10 narrow > $o/hwq$q.log 2>&1 || exit $?
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $o/prof -o fresh -- python3 -u tools/fresh_group_prof.py c2 8 narrow > $o/prof.log 2>&1 || exit $?
exit 0
