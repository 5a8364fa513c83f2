# r3 v8: default bench (with CPU baselines), rocprof kernel trace, PMC traffic C2 / C4
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3v8; mkdir -p $o
timeout -k 10 400 python bench.py > $o/bench.log 2>&1 || exit $?
bash tools/prof_session.sh r3v8/prof > $o/prof.log 2>&1 || exit $?
bash tools/pmc_session.sh r3v8/pmc_c2 > $o/pmc_c2.log 2>&1 || exit $?
bash tools/pmc_session.sh r3v8/pmc_c4 --workload c4 > $o/pmc_c4.log 2>&1 || exit $?
