#!/bin/bash
# rocprofv3 kernel-trace summaries of the end-to-end Resolve (tools/e2e_group_prof.py: bench.py's
# end_to_end block alone -- narrow pinned host shards -> mxp_group_upload2 + mxp_group_resolve_uploaded,
# single calls then the pipelined loop), one process per workload:
# gpurun_out/$1/kernel_stats_e2e_<w>.csv (the pack, evaluation, resolve and copy kernels of the calls).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1
shift
mkdir -p "$out"
for w in "$@"; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/e2e_$w" -o run -- \
        python3 tools/e2e_group_prof.py $w 3 > "$out/e2e_$w.log" 2>&1
    rc=$?
    echo "rocprof e2e $w rc=$rc"
    [ $rc -ne 0 ] && exit $rc
    find "$out/e2e_$w" -name "*kernel_stats.csv" -exec cp {} "$out/kernel_stats_e2e_$w.csv" \;
done
exit 0
