# round-3 final checkpoint at HEAD: GPU suite, smoke, default bench (+ c4 block), C5-quota bench,
# rocprof trace, PMC C2 / C4, SQ counters C2 / C4
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3f2; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
bash tools/prof_session.sh r3f2/prof > $o/prof.log 2>&1 || exit $?
bash tools/pmc_session.sh r3f2/pmc_c2 > $o/pmc_c2.log 2>&1 || exit $?
bash tools/pmc_session.sh r3f2/pmc_c4 --workload c4 > $o/pmc_c4.log 2>&1 || exit $?
bash tools/sq_session.sh r3f2/sq_c2 > $o/sq_c2.log 2>&1 || exit $?
bash tools/sq_session.sh r3f2/sq_c4 --workload c4 > $o/sq_c4.log 2>&1 || exit $?
