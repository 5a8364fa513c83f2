#!/bin/bash
# Copy a closing run's summaries (tools/sessions/r6_final{7,8}.sh -> gpurun_out/<run>) into profiles/:
# fingerprinted HBM traffic and SQ counters (read by bench.py), SQ tables, per-workload and end-to-end
# kernel tables, the GPU suite / smoke / bench logs.
#   bash tools/install_closing.sh r6i
set -eu
cd "$(dirname "$0")/.."
src=gpurun_out/$1
p=profiles
for w in c2 c4 c5 c3-ip c3-str c3-regex; do
    j=$(ls $src/pmc_$w/pmc_traffic_*.json)
    cp "$j" $p/
done
for w in c2 c4 c3-ip c3-str c3-regex; do
    cp $src/sq_$w/sq_counters.json $p/sq_counters_$w.json
    cp $src/sq_$w/sq_table.txt $p/r6_final_sq_table_$w.txt
done
for w in c2 c4 c5 c3-ip c3-str c3-regex e2e_c2 e2e_c4; do
    cp $src/prof/kernel_stats_$w.csv $p/r6_final_kernel_stats_$w.csv
done
cp $src/prof/e2e_c2.log $p/r6_final_e2e_c2.log
cp $src/prof/e2e_c4.log $p/r6_final_e2e_c4.log
cp $src/t.log $p/r6_final_gpu_tests.log
cp $src/smoke.log $p/r6_final_smoke.log
cp $src/bench.log $p/r6_final_bench_default.log
cp $src/fingerprint.txt $p/r6_final_fingerprint.txt
echo installed from $src
