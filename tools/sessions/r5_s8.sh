# round 5, session 8: pointer attributes of pinned memory; the C2 / C4 traces with the download
# paths printed; A/B of the chunked prefix probes (ablib builds) on C2 and C4.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s8; mkdir -p $o
timeout -k 10 60 tools/ptr_probe > $o/ptr.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/e2e_trace.py --workload c2 --reps 2 > $o/e2e_c2.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/e2e_trace.py --workload c4 --reps 2 > $o/e2e_c4.log 2>&1 || exit $?
for wl in c4 c2; do
  for k in 1 2; do
    for lib in "" ablib/libmxp_kc2w6.so ablib/libmxp_kc2w5.so ablib/libmxp_kc4w4.so ablib/libmxp_kc4w5.so; do
      echo "lib ${lib:-in-tree}" >> $o/ab_probe_$wl.log
      MXP_LIB=$lib timeout -k 10 200 python -u tools/steady.py $wl "" >> $o/ab_probe_$wl.log 2>&1 || exit $?
    done
  done
done
