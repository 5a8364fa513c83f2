# round-3 checkpoint at HEAD: GPU suite, smoke, default bench, rocprof trace, PMC C2 / C4
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3fin; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
bash tools/prof_session.sh r3fin/prof > $o/prof.log 2>&1 || exit $?
bash tools/pmc_session.sh r3fin/pmc_c2 > $o/pmc_c2.log 2>&1 || exit $?
bash tools/pmc_session.sh r3fin/pmc_c4 --workload c4 > $o/pmc_c4.log 2>&1 || exit $?
