# round 5, session 6: host link rates (DMA each way, both at once, kernel loads/stores to mapped
# host memory; SDMA on and off), the C2 trace with the pack / error-record / resolve sub-phases
# (columns copied after the strings, the default, and beside them), pipelined end-to-end Resolve
# with 1..3 engines, and the row-N1 ablation on the current C4 build (no rule DFA walk; results
# invalid) alternated with the in-tree library.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s6; mkdir -p $o
timeout -k 10 120 tools/pcie_probe > $o/pcie.log 2>&1 || exit $?
HSA_ENABLE_SDMA=0 timeout -k 10 120 tools/pcie_probe > $o/pcie_nosdma.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/e2e_trace.py --workload c2 > $o/e2e_c2.log 2>&1 || exit $?
MXP_PACK_COLS_BESIDE=1 timeout -k 10 200 python -u tools/e2e_trace.py --workload c2 > $o/e2e_c2_beside.log 2>&1 || exit $?
for k in 1 2; do
  timeout -k 10 200 python -u tools/steady.py c4 "" >> $o/ab_n1_nodfa_c4.log 2>&1 || exit $?
  MXP_LIB=ablib/libmxp_r5_nodfa.so timeout -k 10 200 python -u tools/steady.py c4 "" >> $o/ab_n1_nodfa_c4.log 2>&1 || exit $?
done
timeout -k 10 300 python -u tools/e2e_pipe.py --workload c2 --engines 3 --calls 8 > $o/pipe_c2.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/e2e_pipe.py --workload c4 --engines 2 --calls 4 > $o/pipe_c4.log 2>&1 || exit $?
