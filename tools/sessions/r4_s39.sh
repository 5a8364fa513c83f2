#!/bin/bash
# round 4, session 39: the sort kernel takes four lists as one range of entries; builds alternated, C4,
# 20 evaluations back to back; GPU suite on the variant
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s39; mkdir -p $o
AB_LOOP=20 AB_COMPACT=1 tools/ab_libs.sh c4 ablib/libmxp_r4s39head.so ablib/libmxp_r4s39flat.so > $o/ab_c4.log 2>&1 || exit $?
AB_LOOP=20 AB_COMPACT=1 tools/ab_libs.sh c2 ablib/libmxp_r4s39head.so ablib/libmxp_r4s39flat.so > $o/ab_c2.log 2>&1 || exit $?
grep -v amdgpu.ids $o/ab_c4.log $o/ab_c2.log
MXP_LIB=ablib/libmxp_r4s39flat.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -2 $o/gpu_tests.log
