# round 5, session 12: A/B of the value-class fill's staged gathers (four groups per ds_read_b128,
# unrolled / rolled) against the in-tree layout on C4, processes alternated; parity of the variants.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s12; mkdir -p $o
for k in 1 2; do
  for lib in "" ablib/libmxp_vti1.so ablib/libmxp_vti2.so; do
    echo "lib ${lib:-in-tree}" >> $o/ab_vti_c4.log
    MXP_LIB=$lib timeout -k 10 200 python -u tools/steady.py c4 "" >> $o/ab_vti_c4.log 2>&1 || exit $?
  done
done
for lib in ablib/libmxp_vti1.so ablib/libmxp_vti2.so; do
  MXP_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_vt.py -m gpu -x -q \
    --timeout 200 --timeout-method thread >> $o/t_vti.log 2>&1 || exit $?
done
