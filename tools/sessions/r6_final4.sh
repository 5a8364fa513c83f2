# round 6, final session 4 (after the count-pass change): traffic and SQ counters of the C3 lists, the per-workload kernel tables,
# the end-to-end kernel tables, the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6g; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib2.sha1
for w in c3-ip c3-str c3-regex; do
    bash tools/pmc_session.sh r6g/pmc_$w --workload $w --gen-procs 1 > $o/pmc_$w.log 2>&1 || exit $?
    bash tools/sq_session.sh r6g/sq_$w --workload $w --gen-procs 1 > $o/sq_$w.log 2>&1 || exit $?
    python3 tools/sq_summarize.py gpurun_out/r6g/sq_$w --workload $w > $o/sq_sum_$w.log 2>&1 || exit $?
done
bash tools/prof_workloads.sh r6g/prof --gen-procs 1 > $o/prof.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 bash tools/prof_e2e.sh r6g/prof c2 c4 > $o/prof_e2e.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > $o/bench.log 2>&1 || exit $?
# the driver's N > 1 launch, rehearsed on one GPU: rank 0 drives a two-member group over device 0
# (host reduction), rank 1 waits at the gloo barrier
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --devices 0,0 --steps 10 --warmup 3 --no-cpu-baseline --no-c3 > $o/bench_launch2.log 2>&1 || exit $?
exit 0
