# round 4, session 7: the GPU suite on the in-tree build (two-level class dictionary, fixed word-wise
# interning, literal-key postings), the default bench line with its CPU baselines, rocprof summary
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s7; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $o/bench.json 2> $o/bench.err || exit $?
bash tools/prof_session.sh r4s7/prof --no-c3 > $o/prof.log 2>&1 || exit $?
AB_COMPACT=1 timeout -k 10 300 python tools/ab.py c4 "" "MXP_DEBUG_FLAGS=1024" > $o/ab_c4_probes_only.log 2>&1 || exit $?
WT_COMPACT=1 timeout -k 10 300 python tools/wave_times.py > $o/wave_times_c4.log 2>&1 || exit $?
