# round 6, final session 7 (after the pair Resolve): the whole GPU suite and smoke on the final build, then the HBM traffic
# (FETCH / WRITE passes) and SQ counters of C2, C4 and C5 (one data-generating process: the
# profiler's preload initialises the GPU before bench.py's fork pool would run).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6i; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib.sha1
python3 -c "import bench; print(bench.kernel_fingerprint())" > $o/fingerprint.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
bash tools/pmc_session.sh r6i/pmc_c2 --gen-procs 1 > $o/pmc_c2.log 2>&1 || exit $?
bash tools/pmc_session.sh r6i/pmc_c4 --workload c4 --gen-procs 1 > $o/pmc_c4.log 2>&1 || exit $?
bash tools/pmc_session.sh r6i/pmc_c5 --workload c5 --gen-procs 1 > $o/pmc_c5.log 2>&1 || exit $?
bash tools/sq_session.sh r6i/sq_c2 --gen-procs 1 > $o/sq_c2.log 2>&1 || exit $?
python3 tools/sq_summarize.py gpurun_out/r6i/sq_c2 --workload c2 > $o/sq_sum_c2.log 2>&1 || exit $?
bash tools/sq_session.sh r6i/sq_c4 --workload c4 --gen-procs 1 > $o/sq_c4.log 2>&1 || exit $?
python3 tools/sq_summarize.py gpurun_out/r6i/sq_c4 --workload c4 > $o/sq_sum_c4.log 2>&1 || exit $?
exit 0
