#!/bin/bash
# round 4, session 26: guard-index load factor past the old clamp (MXP_INDEX_SPARSITY 5..8)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s26; mkdir -p $o
AB_COMPACT=1 timeout -k 10 300 python tools/ab.py c4 "" "MXP_INDEX_SPARSITY=4" "MXP_INDEX_SPARSITY=5" "MXP_INDEX_SPARSITY=6" "MXP_INDEX_SPARSITY=8" > $o/ab_c4_sparsity.log 2>&1 || exit $?
AB_COMPACT=1 timeout -k 10 300 python tools/ab.py c2 "" "MXP_INDEX_SPARSITY=4" "MXP_INDEX_SPARSITY=5" "MXP_INDEX_SPARSITY=6" > $o/ab_c2_sparsity.log 2>&1 || exit $?
grep -v amdgpu.ids $o/ab_c4_sparsity.log $o/ab_c2_sparsity.log
