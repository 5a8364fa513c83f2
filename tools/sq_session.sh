#!/bin/bash
# SQ counters of the bench's kernels (issue / wait breakdown, instruction mix, LDS bank conflicts),
# one rocprofv3 --pmc pass per group (SQ has 8 slots per pass on gfx950), each under its own limit.
#   bash tools/sq_session.sh <outdir> [bench args]     (per workload: C2 alone, or --workload c4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1
shift
mkdir -p "$out"
passes=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
  "SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"
)
i=0
for p in "${passes[@]}"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d "$out/sq$i" -o pmc -- \
        python3 bench.py --no-cpu-baseline --no-c4 --no-c5 --no-c3 --fresh-steps 0 --e2e-reps 0 --steps 2 --warmup 1 "$@" > "$out/sq$i.log" 2>&1
    rc=$?
    echo "sq$i rc=$rc"
    [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_table.py "$out"/sq* > "$out/sq_table.txt"
cat "$out/sq_table.txt"
