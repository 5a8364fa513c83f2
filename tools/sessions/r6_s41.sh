# round 6, session 41: why the bench's pipelined C2 end-to-end period (2.41 ms in the closing line)
# is slower than the same function run alone (1.78 ms, tools/e2e_group_prof.py): the tool, then the
# C2 block alone with and without the fresh-batch block before it
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s41; mkdir -p $o
timeout -k 10 200 python -u tools/e2e_group_prof.py c2 3 > $o/tool.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-c3 --no-c4 --no-c5 --no-cpu-baseline > $o/bench_c2.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-c3 --no-c4 --no-c5 --no-cpu-baseline --fresh-steps 0 > $o/bench_c2_nofresh.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-c3 --no-c4 --no-c5 --no-cpu-baseline --steps 0 --warmup 0 > $o/bench_c2_nosteps.log 2>&1
echo "nosteps rc=$?" >> $o/bench_c2_nosteps.log
exit 0
