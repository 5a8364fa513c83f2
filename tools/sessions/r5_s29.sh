# round 5, session 29: the fast/slow fill split's parity test (in-tree, closing build), then the
# fast fill's pair test hoisted ahead of the merge loop (ablib hoist) against the in-tree build,
# C4 steady state alternated.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s29; mkdir -p $o
sha1sum istio_amd/libmxp.so ablib/*.so > $o/libs.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_vtfill_split.py -m gpu -x -v \
  --timeout 200 --timeout-method thread > $o/t.log 2>&1 || exit $?
for k in 1 2 3; do
  for lib in "" ablib/libmxp_hoist.so; do
    echo "lib ${lib:-in-tree}" >> $o/ab_c4.log
    MXP_LIB=$lib timeout -k 10 200 python -u tools/steady.py c4 "" >> $o/ab_c4.log 2>&1 || exit $?
  done
done
