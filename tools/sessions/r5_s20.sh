# round 5, session 20: value-class fill with the group loop unrolled at compile time (immediate
# LDS offsets, one-compare pair test, scalar row bases; errors on the general loop) -- in-tree --
# against the round-5 closing build (ablib r5base) and the same capped at 4 waves/SIMD (ablib
# vtfw4), C4 steady state alternated; then the value-class / deferred-pair parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s20; mkdir -p $o
sha1sum istio_amd/libmxp.so ablib/*.so > $o/libs.txt
for k in 1 2; do
  for lib in ablib/libmxp_r5base.so "" ablib/libmxp_vtfw4.so; do
    echo "lib ${lib:-in-tree}" >> $o/ab_c4.log
    MXP_LIB=$lib timeout -k 10 200 python -u tools/steady.py c4 "" >> $o/ab_c4.log 2>&1 || exit $?
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_vt.py tests/test_gpu_dtp.py tests/test_gpu_scale.py -m gpu -x -v \
  --timeout 200 --timeout-method thread > $o/t.log 2>&1 || exit $?
