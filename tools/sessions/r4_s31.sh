#!/bin/bash
# round 4, session 31: the prefix hash keeps the string word it loaded (one load per 8 bytes of
# the request's string instead of one per probed key length); same-box A/B against HEAD's build,
# C4 and C2, back-to-back evaluations; GPU suite on the variant
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s31; mkdir -p $o
AB_LOOP=20 AB_COMPACT=1 tools/ab_libs.sh c4 ablib/libmxp_r4s31head.so ablib/libmxp_r4s31word.so > $o/ab_c4.log 2>&1 || exit $?
AB_LOOP=20 AB_COMPACT=1 tools/ab_libs.sh c2 ablib/libmxp_r4s31head.so ablib/libmxp_r4s31word.so > $o/ab_c2.log 2>&1 || exit $?
grep -v amdgpu.ids $o/ab_c4.log $o/ab_c2.log
MXP_LIB=ablib/libmxp_r4s31word.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -2 $o/gpu_tests.log
