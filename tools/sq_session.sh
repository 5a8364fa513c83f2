#!/bin/bash
# SQ counters (issue / wait breakdown, instruction mix) of the bench's kernels in one rocprofv3
# --pmc pass (SQ has 8 slots on gfx950); counter list first, for reference.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1
shift
mkdir -p "$out"
timeout -k 10 120 rocprofv3 -L > "$out/counters.txt" 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
    --output-format csv -d "$out/sq1" -o pmc -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" > "$out/sq1.log" 2>&1
rc=$?; echo "sq1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_SENDMSG SQ_INST_CYCLES_SALU \
    --output-format csv -d "$out/sq2" -o pmc -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" > "$out/sq2.log" 2>&1
rc=$?; echo "sq2 rc=$rc"
exit $rc
