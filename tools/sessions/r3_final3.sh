# round-3 closing session at HEAD: GPU suite, smoke, PMC C2 / C4 of this build, then the default
# bench line (its roofline carries this build's PMC traffic) and the rocprof trace
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3f3; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
bash tools/pmc_session.sh r3f3/pmc_c2 > $o/pmc_c2.log 2>&1 || exit $?
bash tools/pmc_session.sh r3f3/pmc_c4 --workload c4 > $o/pmc_c4.log 2>&1 || exit $?
python3 tools/pmc_summarize.py gpurun_out/r3f3/pmc_c2 --workload c2 > $o/pmc_sum_c2.log 2>&1 && cp gpurun_out/r3f3/pmc_c2/pmc_traffic_c2.json profiles/ || exit $?
python3 tools/pmc_summarize.py gpurun_out/r3f3/pmc_c4 --workload c4 > $o/pmc_sum_c4.log 2>&1 && cp gpurun_out/r3f3/pmc_c4/pmc_traffic_c4.json profiles/ || exit $?
timeout -k 10 400 python -u bench.py > $o/bench.log 2>&1 || exit $?
bash tools/prof_session.sh r3f3/prof > $o/prof.log 2>&1 || exit $?
