#!/bin/bash
# round 4, session 23: compare continuations evaluated without the interpreter (mxp_tmpl.simple):
# GPU suite on the new build, then same-box A/B against HEAD's build on C2 and C4
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s23; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -3 $o/gpu_tests.log
AB_COMPACT=1 tools/ab_libs.sh c2 ablib/libmxp_r4s23head.so ablib/libmxp_r4s23simple.so > $o/ab_c2.log 2>&1 || exit $?
AB_COMPACT=1 tools/ab_libs.sh c4 ablib/libmxp_r4s23head.so ablib/libmxp_r4s23simple.so > $o/ab_c4.log 2>&1 || exit $?
cat $o/ab_c2.log $o/ab_c4.log
