# round 4, session 4: immediate-offset value-class fill (mxp_vtfill_imm<n>_kernel) + vt_mark word
# pooling; tests, same-box A/B against the round-start build, rocprof stats of the bench
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r4s4; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_vt.py tests/test_gpu_pack.py tests/test_gpu_dtp.py tests/test_gpu_scale.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $o/t.log 2>&1 || exit $?
AB_COMPACT=1 bash tools/ab_libs.sh c4 ablib/libmxp_base.so ablib/libmxp_r4b.so > $o/ab_c4.log 2>&1 || exit $?
bash tools/prof_session.sh r4s4/prof > $o/prof.log 2>&1 || exit $?
