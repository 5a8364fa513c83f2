# round 6, session 12: counters of the C3 regex kernel with prefix dispatch (issue / wait mix, L2 hits)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s12; mkdir -p $o
bash tools/sq_session.sh r6s12/sq --workload c3-regex --gen-procs 1 > $o/sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d $o/tcc -o pmc -- python3 bench.py --no-cpu-baseline --fresh-steps 0 --e2e-reps 0 --steps 2 --warmup 1 --workload c3-regex --gen-procs 1 > $o/tcc.log 2>&1 || exit $?
python3 tools/pmc_table.py $o/tcc > $o/tcc_table.txt
exit 0
