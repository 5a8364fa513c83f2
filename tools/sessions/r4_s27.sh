#!/bin/bash
# round 4, session 27: guard-index tables at 64 slots per key by default (index_sparsity 5): GPU
# suite, then same-box A/B against HEAD's build (2^3 slots per key) on C4 and C2
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s27; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -2 $o/gpu_tests.log
AB_COMPACT=1 tools/ab_libs.sh c4 ablib/libmxp_head.so ablib/libmxp_r4s27s5.so > $o/ab_c4.log 2>&1 || exit $?
AB_COMPACT=1 tools/ab_libs.sh c2 ablib/libmxp_head.so ablib/libmxp_r4s27s5.so > $o/ab_c2.log 2>&1 || exit $?
grep -v amdgpu.ids $o/ab_c4.log $o/ab_c2.log
