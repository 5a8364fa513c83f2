# round 6, session 28: four members on device 0 through the whole bench (the 8-GPU group's code
# paths with more members than two: rendezvous, host reduction, owner routing of 4 shards)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s28; mkdir -p $o
MXP_BENCH_WATCHDOG=150 timeout -k 10 700 python -u bench.py --devices 0,0,0,0 --steps 5 --warmup 2 --no-cpu-baseline > $o/bench4.log 2> $o/bench4.err
echo "rc=$?" >> $o/bench4.err
exit 0
