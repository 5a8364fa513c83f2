#!/bin/bash
# round 4, session 32: engine knobs re-swept on this build (settings alternated in one process, 20
# evaluations back to back): fill chunk 8 / 12 groups, deferred-pair list 1024 / 4096 per wave, C2
# fill span 2 / 8
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s32; mkdir -p $o
AB_LOOP=20 AB_COMPACT=1 timeout -k 10 400 python tools/ab.py c4 "" "MXP_FILL_CHUNK=8" "MXP_FILL_CHUNK=12" "MXP_DTP_CAP=1024" "MXP_DTP_CAP=4096" > $o/ab_c4.log 2>&1 || exit $?
AB_LOOP=20 AB_COMPACT=1 timeout -k 10 400 python tools/ab.py c2 "" "MXP_FILL_CHUNK=8" "MXP_DTP_CAP=1024" "MXP_DTP_CAP=4096" "MXP_FILL_SPAN=2" "MXP_FILL_SPAN=8" > $o/ab_c2.log 2>&1 || exit $?
grep -v amdgpu.ids $o/ab_c4.log $o/ab_c2.log
