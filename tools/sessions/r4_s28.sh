#!/bin/bash
# round 4, session 28: the engine's ordering events (deferred-pair, hit-counter gate, chunk events)
# recorded without a system-scope fence; same-box A/B against HEAD's build, single evaluations and
# 20 back to back (the bench's loop), C2 and C4; then the GPU suite on the new build
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s28; mkdir -p $o
AB_LOOP=20 AB_COMPACT=1 tools/ab_libs.sh c2 ablib/libmxp_r4s27s5.so ablib/libmxp_r4s28ev.so > $o/ab_c2_loop.log 2>&1 || exit $?
AB_LOOP=20 AB_COMPACT=1 tools/ab_libs.sh c4 ablib/libmxp_r4s27s5.so ablib/libmxp_r4s28ev.so > $o/ab_c4_loop.log 2>&1 || exit $?
AB_COMPACT=1 tools/ab_libs.sh c2 ablib/libmxp_r4s27s5.so ablib/libmxp_r4s28ev.so > $o/ab_c2.log 2>&1 || exit $?
grep -v amdgpu.ids $o/ab_c2_loop.log $o/ab_c4_loop.log $o/ab_c2.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -2 $o/gpu_tests.log
