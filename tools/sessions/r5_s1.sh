# round 5, session 1: GPU suite (batch validation, bin cap, free-after-stream-destroy), smoke, C3
# PMC + SQ counters per list kind, per-workload kernel tables, default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s1; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
for w in c3-ip c3-str c3-regex; do
    bash tools/pmc_session.sh r5s1/pmc_$w --workload $w > $o/pmc_$w.log 2>&1 || exit $?
    bash tools/sq_session.sh r5s1/sq_$w --workload $w > $o/sq_$w.log 2>&1 || exit $?
    python3 tools/sq_summarize.py gpurun_out/r5s1/sq_$w --workload $w > $o/sq_sum_$w.log 2>&1 || exit $?
done
bash tools/prof_workloads.sh r5s1/prof > $o/prof.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > $o/bench.log 2>&1 || exit $?
