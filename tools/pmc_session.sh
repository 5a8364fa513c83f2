#!/bin/bash
# HBM traffic of the bench's evaluation kernels: FETCH_SIZE and WRITE_SIZE in separate rocprofv3
# --pmc passes (they do not fit one TCC pass on gfx950), then tools/pmc_summarize.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1
shift
mkdir -p "$out"
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$out/$c" -o pmc -- \
        python3 bench.py --no-cpu-baseline --no-c4 --no-c5 --no-c3 --fresh-steps 0 --e2e-reps 0 --steps 3 --warmup 1 "$@" > "$out/$c.log" 2>&1
    rc=$?
    echo "pmc $c rc=$rc"
    [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_summarize.py "$out" "$@"
