#!/bin/bash
# round 4, session 24: the deferred-pair sort's partial-line slot stores -- a capped grid (tiles
# taken in grid stride, so fewer tiles' slot rows are open in L2 at once) and a smaller chunk window;
# GPU suite on the capped-grid build, same-box A/B against HEAD's build, PMC WRITE_SIZE per build
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s24; mkdir -p $o
MXP_LIB=ablib/libmxp_r4s24g256.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests_g256.log 2>&1 || { tail -30 $o/gpu_tests_g256.log; exit 1; }
tail -2 $o/gpu_tests_g256.log
for v in g256 g512 win8; do
    AB_COMPACT=1 tools/ab_libs.sh c4 ablib/libmxp_head.so ablib/libmxp_r4s24$v.so > $o/ab_c4_$v.log 2>&1 || exit $?
    grep -v amdgpu.ids $o/ab_c4_$v.log
done
AB_COMPACT=1 tools/ab_libs.sh c2 ablib/libmxp_head.so ablib/libmxp_r4s24g256.so > $o/ab_c2_g256.log 2>&1 || exit $?
grep -v amdgpu.ids $o/ab_c2_g256.log
for v in head r4s24g256 r4s24g512 r4s24win8; do
    MXP_LIB=ablib/libmxp_$v.so AB_COMPACT=1 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/pmc_$v -o pmc -- python3 tools/ab.py c4 "" > $o/pmc_$v.log 2>&1 || { echo "pmc $v rc=$?"; exit 1; }
    MXP_LIB=ablib/libmxp_$v.so AB_COMPACT=1 timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $o/kt_$v -o kt -- python3 tools/ab.py c4 "" > $o/kt_$v.log 2>&1 || { echo "kt $v rc=$?"; exit 1; }
done
echo done
