# round 5, session 18: A/B of the index kernels loading a request's string head without waiting
# for its kinds (MXP_HEAD_EARLY=1, ablib) against the in-tree library, C2 and C4, alternated.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s18; mkdir -p $o
for wl in c2 c4; do
  for k in 1 2 3; do
    for lib in "" ablib/libmxp_headearly.so; do
      echo "lib ${lib:-in-tree}" >> $o/ab_head_$wl.log
      MXP_LIB=$lib timeout -k 10 200 python -u tools/steady.py $wl "" >> $o/ab_head_$wl.log 2>&1 || exit $?
    done
  done
done
MXP_LIB=ablib/libmxp_headearly.so timeout -k 10 300 python -u -m pytest tests/test_gpu_heads.py tests/test_gpu_scale.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > $o/t.log 2>&1 || exit $?
