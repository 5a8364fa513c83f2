#!/bin/bash
# round 4, session 35: the per-wave deferred-pair list stride -- 2048 entries (8 KB, a power of two:
# the sort kernel's four concurrent list reads alias) against odd multiples of 128 bytes
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s35; mkdir -p $o
AB_LOOP=20 AB_COMPACT=1 timeout -k 10 400 python tools/ab.py c4 "" "MXP_DTP_CAP=2080" "MXP_DTP_CAP=2016" "MXP_DTP_CAP=1792" > $o/ab_c4.log 2>&1 || exit $?
AB_LOOP=20 AB_COMPACT=1 timeout -k 10 400 python tools/ab.py c4p "" "MXP_DTP_CAP=2080" "MXP_DTP_CAP=2016" > $o/ab_c4p.log 2>&1 || exit $?
grep -v amdgpu.ids $o/ab_c4.log $o/ab_c4p.log
