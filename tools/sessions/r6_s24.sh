# round 6, session 24: a two-member group on device 0 through the whole bench (no launcher), with
# Python stacks every 45 s, to find where the rehearsed N = 2 launch stopped
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s24; mkdir -p $o
MXP_BENCH_WATCHDOG=45 timeout -k 10 200 python -u bench.py --devices 0,0 --steps 5 --warmup 2 --no-cpu-baseline --no-c3 > $o/bench.log 2> $o/bench.err
echo "rc=$?" >> $o/bench.err
exit 0
