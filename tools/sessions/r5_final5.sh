# round-5 closing session (after the value-class fill split), part 1: the new
# tests and the fresh-batch timeline first, then the whole GPU suite, smoke, PMC traffic (C2, C4,
# C5) and SQ counters (C2, C4) of this build.  Summaries land in gpurun_out/r5h.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5h; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib.sha1
timeout -k 10 600 python -u -m pytest tests/test_gpu_async_upload.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $o/t_new.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $o/fresh_c2 -o run -- \
  python3 tools/fresh_prof.py c2 8 > $o/fresh_c2.log 2>&1 || exit $?
python3 tools/copy_timeline.py $o/fresh_c2 4 > $o/timeline_c2.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
bash tools/pmc_session.sh r5h/pmc_c2 > $o/pmc_c2.log 2>&1 || exit $?
bash tools/pmc_session.sh r5h/pmc_c4 --workload c4 > $o/pmc_c4.log 2>&1 || exit $?
bash tools/pmc_session.sh r5h/pmc_c5 --workload c5 > $o/pmc_c5.log 2>&1 || exit $?
bash tools/sq_session.sh r5h/sq_c2 > $o/sq_c2.log 2>&1 || exit $?
python3 tools/sq_summarize.py gpurun_out/r5h/sq_c2 --workload c2 > $o/sq_sum_c2.log 2>&1 || exit $?
bash tools/sq_session.sh r5h/sq_c4 --workload c4 > $o/sq_c4.log 2>&1 || exit $?
python3 tools/sq_summarize.py gpurun_out/r5h/sq_c4 --workload c4 > $o/sq_sum_c4.log 2>&1 || exit $?
