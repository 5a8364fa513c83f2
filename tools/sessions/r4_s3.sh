# round 4, session 3: vt_mark dedup (upload) + branch-free staged vtfill per active-slot count;
# tests, same-box A/B against the round-start build, bench line (fresh-batch block), rocprof stats
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r4s3; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_vt.py tests/test_gpu_pack.py tests/test_gpu_dtp.py tests/test_gpu_scale.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $o/t.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_base.so ablib/libmxp_r4a.so > $o/ab_c4.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c2 ablib/libmxp_base.so ablib/libmxp_r4a.so > $o/ab_c2.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $o/bench.log 2>&1 || exit $?
bash tools/prof_session.sh r4s3/prof > $o/prof.log 2>&1 || exit $?
