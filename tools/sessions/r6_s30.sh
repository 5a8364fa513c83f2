# round 6, session 30: the single end-to-end call with the upload not waiting for its copies
# (MXP_UPLOAD_NO_WAIT, default now) against waiting (BENCH_E2E_WAIT=1), alternated
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1 GPU_MAX_HW_QUEUES=8
o=gpurun_out/r6s30; mkdir -p $o
for rep in 1 2 3; do
  for w in "" 1; do
    echo "wait=${w:-0}" >> $o/ab.log
    BENCH_E2E_WAIT=$w timeout -k 10 200 python -u tools/e2e_group_prof.py c2 5 2>&1 | grep ms_per_batch >> $o/ab.log || exit $?
  done
done
exit 0
