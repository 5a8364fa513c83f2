#!/bin/bash
# round 4, session 37: value-class index rows padded off 2^k (MXP_VT_PITCH); builds alternated, C4,
# 20 evaluations back to back; GPU suite on the variant
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s37; mkdir -p $o
AB_LOOP=20 AB_COMPACT=1 tools/ab_libs.sh c4 ablib/libmxp_r4s37head.so ablib/libmxp_r4s37pitch.so > $o/ab_c4.log 2>&1 || exit $?
grep -v amdgpu.ids $o/ab_c4.log
MXP_LIB=ablib/libmxp_r4s37pitch.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -2 $o/gpu_tests.log
