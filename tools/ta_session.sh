#!/bin/bash
# TA / TD / TCP counters of the bench's kernels (address-unit busy, TLB hits and misses, L1 -> L2
# read requests and their latency), one rocprofv3 --pmc pass per group (2 TA, 2 TD, 4 TCP slots).
#   bash tools/ta_session.sh <outdir> [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1
shift
mkdir -p "$out"
passes=(
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE"
  "TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_ADDR_STALL_CYCLES_sum TCP_UTCL1_STALL_MULTI_MISS_sum"
)
i=0
for p in "${passes[@]}"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d "$out/ta$i" -o pmc -- \
        python3 bench.py --no-cpu-baseline --e2e-reps 0 --steps 2 --warmup 1 "$@" > "$out/ta$i.log" 2>&1
    rc=$?
    echo "ta$i rc=$rc"
    [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_table.py "$out"/ta* > "$out/ta_table.txt"
cat "$out/ta_table.txt"
