# round 5, session 23: tiles of 1024 requests per value-class fill workgroup (MXP_VTF_TILES 4,
# in-tree, against 2 and 8, ablib vtft2 / vtft8), C4 steady state alternated; SQ counters of the
# split fill (in-tree).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s23; mkdir -p $o
sha1sum istio_amd/libmxp.so ablib/*.so > $o/libs.txt
for k in 1 2; do
  for lib in "" ablib/libmxp_vtft2.so ablib/libmxp_vtft8.so; do
    echo "lib ${lib:-in-tree}" >> $o/ab_c4.log
    MXP_LIB=$lib timeout -k 10 200 python -u tools/steady.py c4 "" >> $o/ab_c4.log 2>&1 || exit $?
  done
done
bash tools/sq_session.sh r5s23/sq --workload c4 > $o/sq.log 2>&1 || exit $?
