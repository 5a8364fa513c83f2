# r3 v2: heads GPU test, default bench, rocprof kernel trace, PMC traffic C2 / C4
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3v2; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_heads.py -x -q --timeout 200 --timeout-method thread > $o/heads.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $o/bench.log 2>&1 || exit $?
bash tools/prof_session.sh r3v2/prof > $o/prof.log 2>&1 || exit $?
bash tools/pmc_session.sh r3v2/pmc_c2 > $o/pmc_c2.log 2>&1 || exit $?
bash tools/pmc_session.sh r3v2/pmc_c4 --workload c4 > $o/pmc_c4.log 2>&1 || exit $?
AB_COMPACT=1 timeout -k 10 200 python tools/ab.py c4 MXP_DEBUG_FLAGS=0 MXP_DEBUG_FLAGS=4194304 > $o/ab_c4_vtcount.log 2>&1 || exit $?
