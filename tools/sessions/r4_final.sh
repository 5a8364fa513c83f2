# round-4 closing session at HEAD: GPU suite, smoke, PMC traffic (C2, C4, C5) and SQ counters (C2,
# C4) of this build, then the default bench line and the rocprof summary.  The summaries land in
# gpurun_out/r4f and are copied into profiles/ by hand after the call.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4f; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
bash tools/pmc_session.sh r4f/pmc_c2 > $o/pmc_c2.log 2>&1 || exit $?
bash tools/pmc_session.sh r4f/pmc_c4 --workload c4 > $o/pmc_c4.log 2>&1 || exit $?
bash tools/pmc_session.sh r4f/pmc_c5 --workload c5 > $o/pmc_c5.log 2>&1 || exit $?
bash tools/sq_session.sh r4f/sq_c2 > $o/sq_c2.log 2>&1 || exit $?
python3 tools/sq_summarize.py gpurun_out/r4f/sq_c2 --workload c2 > $o/sq_sum_c2.log 2>&1 || exit $?
bash tools/sq_session.sh r4f/sq_c4 --workload c4 > $o/sq_c4.log 2>&1 || exit $?
python3 tools/sq_summarize.py gpurun_out/r4f/sq_c4 --workload c4 > $o/sq_sum_c4.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > $o/bench.log 2>&1 || exit $?
bash tools/prof_session.sh r4f/prof > $o/prof.log 2>&1 || exit $?
