#!/bin/bash
# round 4, session 34: deferred-pair list 1280 / 1536 per wave on the pair-dense C4 path routes
# (c4p) and C2, against the 2048 default
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s34; mkdir -p $o
AB_LOOP=20 AB_COMPACT=1 timeout -k 10 400 python tools/ab.py c4p "" "MXP_DTP_CAP=1280" "MXP_DTP_CAP=1536" "MXP_DTP_CAP=1792" > $o/ab_c4p.log 2>&1 || exit $?
AB_LOOP=20 AB_COMPACT=1 timeout -k 10 400 python tools/ab.py c4 "" "MXP_DTP_CAP=1536" "MXP_DTP_CAP=1792" > $o/ab_c4.log 2>&1 || exit $?
AB_LOOP=20 AB_COMPACT=1 timeout -k 10 400 python tools/ab.py c2 "" "MXP_DTP_CAP=1536" > $o/ab_c2.log 2>&1 || exit $?
grep -v amdgpu.ids $o/ab_c4p.log $o/ab_c4.log $o/ab_c2.log
