#!/bin/bash
# round 4, session 33: the deferred-pair list per index wave (MXP_DTP_CAP; pairs past it take the
# overflow list the post-fill index launch ORs in), swept on C4 (and the C4 path-only routes)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s33; mkdir -p $o
AB_LOOP=20 AB_COMPACT=1 timeout -k 10 400 python tools/ab.py c4 "" "MXP_DTP_CAP=512" "MXP_DTP_CAP=768" "MXP_DTP_CAP=1024" "MXP_DTP_CAP=1280" "MXP_DTP_CAP=1536" > $o/ab_c4.log 2>&1 || exit $?
AB_LOOP=20 AB_COMPACT=1 timeout -k 10 400 python tools/ab.py c4p "" "MXP_DTP_CAP=768" "MXP_DTP_CAP=1024" > $o/ab_c4p.log 2>&1 || exit $?
grep -v amdgpu.ids $o/ab_c4.log $o/ab_c4p.log
