# round-5 closing session, part 1 (at HEAD): the whole GPU suite, smoke, PMC traffic (C2, C4, C5)
# and SQ counters (C2, C4) of this build.  Summaries land in gpurun_out/r5f and are copied into
# profiles/ after the call.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5f; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib.sha1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
bash tools/pmc_session.sh r5f/pmc_c2 > $o/pmc_c2.log 2>&1 || exit $?
bash tools/pmc_session.sh r5f/pmc_c4 --workload c4 > $o/pmc_c4.log 2>&1 || exit $?
bash tools/pmc_session.sh r5f/pmc_c5 --workload c5 > $o/pmc_c5.log 2>&1 || exit $?
bash tools/sq_session.sh r5f/sq_c2 > $o/sq_c2.log 2>&1 || exit $?
python3 tools/sq_summarize.py gpurun_out/r5f/sq_c2 --workload c2 > $o/sq_sum_c2.log 2>&1 || exit $?
bash tools/sq_session.sh r5f/sq_c4 --workload c4 > $o/sq_c4.log 2>&1 || exit $?
python3 tools/sq_summarize.py gpurun_out/r5f/sq_c4 --workload c4 > $o/sq_sum_c4.log 2>&1 || exit $?
