# round 6, session 20: fresh-batch and end-to-end (single / pipelined) C2 at 4 and 8 hardware queues,
# with and without the evaluation streams at the greatest priority (MXP_STREAM_PRIO)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s20; mkdir -p $o
for rep in 1 2; do
for q in 4 8; do
  for p in 0 1; do
    echo "hwq $q prio $p" >> $o/ab.log
    GPU_MAX_HW_QUEUES=$q MXP_STREAM_PRIO=$p timeout -k 10 200 python -u tools/fresh_group_prof.py c2 10 narrow 2>&1 | grep ms_per_step >> $o/ab.log || exit $?
    GPU_MAX_HW_QUEUES=$q MXP_STREAM_PRIO=$p timeout -k 10 200 python -u tools/e2e_group_prof.py c2 5 2>&1 | grep ms_per_batch >> $o/ab.log || exit $?
  done
done
done
exit 0
