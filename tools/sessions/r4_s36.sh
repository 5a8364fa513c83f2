#!/bin/bash
# round 4, session 36: deferred-pair chunk rows padded by 8 quads (a row of 2^k quads put every
# chunk's same quads on aliased channels); builds alternated, 20 evaluations back to back; GPU suite
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s36; mkdir -p $o
AB_LOOP=20 AB_COMPACT=1 tools/ab_libs.sh c4 ablib/libmxp_r4s36head.so ablib/libmxp_r4s36row.so > $o/ab_c4.log 2>&1 || exit $?
AB_LOOP=20 AB_COMPACT=1 tools/ab_libs.sh c2 ablib/libmxp_r4s36head.so ablib/libmxp_r4s36row.so > $o/ab_c2.log 2>&1 || exit $?
grep -v amdgpu.ids $o/ab_c4.log $o/ab_c2.log
MXP_LIB=ablib/libmxp_r4s36row.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -2 $o/gpu_tests.log
