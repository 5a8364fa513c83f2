#!/bin/bash
# round 4, session 38: do the batch's 2^k column strides cost anything? (tools/stride_probe.py)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s38; mkdir -p $o
timeout -k 10 400 python tools/stride_probe.py c2 > $o/stride_c2.log 2>&1 || exit $?
timeout -k 10 400 python tools/stride_probe.py c4 > $o/stride_c4.log 2>&1 || exit $?
grep -v amdgpu.ids $o/stride_c2.log $o/stride_c4.log
