#!/bin/bash
# round 4, session 25: GPU suite (oracle value model split, regex rules against Python's re), and the
# guard-index load factor re-measured now that occupancy bitmaps spare empty slots their entry loads
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s25; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -2 $o/gpu_tests.log
AB_COMPACT=1 timeout -k 10 300 python tools/ab.py c4 "" "MXP_INDEX_SPARSITY=3" "MXP_INDEX_SPARSITY=4" "MXP_INDEX_SPARSITY=1" > $o/ab_c4_sparsity.log 2>&1 || exit $?
AB_COMPACT=1 timeout -k 10 300 python tools/ab.py c2 "" "MXP_INDEX_SPARSITY=3" "MXP_INDEX_SPARSITY=4" "MXP_INDEX_SPARSITY=1" > $o/ab_c2_sparsity.log 2>&1 || exit $?
grep -v amdgpu.ids $o/ab_c4_sparsity.log $o/ab_c2_sparsity.log
