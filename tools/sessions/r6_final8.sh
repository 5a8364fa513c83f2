# round 6, final session 8 (after the pair Resolve): traffic and SQ counters of the C3 lists, the per-workload kernel tables,
# the end-to-end kernel tables, the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6i; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib2.sha1
for w in c3-ip c3-str c3-regex; do
    bash tools/pmc_session.sh r6i/pmc_$w --workload $w --gen-procs 1 > $o/pmc_$w.log 2>&1 || exit $?
    bash tools/sq_session.sh r6i/sq_$w --workload $w --gen-procs 1 > $o/sq_$w.log 2>&1 || exit $?
    python3 tools/sq_summarize.py gpurun_out/r6i/sq_$w --workload $w > $o/sq_sum_$w.log 2>&1 || exit $?
done
bash tools/prof_workloads.sh r6i/prof --gen-procs 1 > $o/prof.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 bash tools/prof_e2e.sh r6i/prof c2 c4 > $o/prof_e2e.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > $o/bench.log 2>&1 || exit $?
exit 0
