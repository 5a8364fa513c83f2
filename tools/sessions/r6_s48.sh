# round 6, session 48: the lite index kernel's probe chunk (MXP_PROBE_KC 2 -> 3) and occupancy
# (MXP_LITE_WAVES 5 -> 4) as builds (abvar/), same-box A/B against the in-tree build, processes alternated
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s48; mkdir -p $o
for v in kc3 kc2w4 kc3w4; do
  AB_COMPACT=1 AB_LOOP=20 bash tools/ab_libs.sh c4 istio_amd/libmxp.so abvar/libmxp_$v.so > $o/ab_c4_$v.log 2>&1 || exit $?
done
AB_COMPACT=1 AB_LOOP=20 bash tools/ab_libs.sh c2 istio_amd/libmxp.so abvar/libmxp_kc3.so > $o/ab_c2_kc3.log 2>&1 || exit $?
exit 0
