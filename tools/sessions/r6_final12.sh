# round 6, final session 12: the driver's N > 1 launch rehearsed on the final tree (two ranks under
# torch.distributed.run; rank 0 drives a two-member group on the one GPU, host reduction)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6l; mkdir -p $o
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --devices 0,0 --steps 5 --warmup 2 --no-cpu-baseline > $o/launch2.log 2> $o/launch2.err || exit $?
exit 0
