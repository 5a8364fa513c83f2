# round 5, session 17: the fresh-batch step with the packer's uploads by the copy engine, and by the
# gather kernel at 32 / 128 / 512 workgroups (tools/fresh_prof.py, processes alternated).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s17; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib.sha1
for k in 1 2; do
  for v in "MXP_H2D_DMA=1" "MXP_H2D_GRID=32" "MXP_H2D_GRID=128" "MXP_H2D_GRID=512"; do
    echo "$v" >> $o/ab_h2d.log
    env $v timeout -k 10 200 python3 tools/fresh_prof.py c2 10 >> $o/ab_h2d.log 2>&1 || exit $?
    env $v timeout -k 10 200 python3 tools/fresh_prof.py c4 10 >> $o/ab_h2d.log 2>&1 || exit $?
  done
done
