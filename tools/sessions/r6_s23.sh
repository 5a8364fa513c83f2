# round 6, session 23: the driver's N > 1 launch rehearsed on one GPU (torch.distributed.run x 2:
# rank 0 drives a two-member group over device 0 with the host reduction, rank 1 waits at the gloo
# barrier); progress notes on stderr
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s23; mkdir -p $o
MXP_BENCH_WATCHDOG=100 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --devices 0,0 --steps 10 --warmup 3 --no-cpu-baseline --no-c3 > $o/bench_launch2.log 2> $o/bench_launch2.err; echo "rc=$?" >> $o/bench_launch2.err
exit 0
