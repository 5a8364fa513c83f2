# memquota: parity, bench, per-key replay profile
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3q; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_memquota.py -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c5-quota --no-cpu-baseline > $o/q.log 2>&1 || exit $?
MXP_QUOTA_PROF=$o/prof.txt timeout -k 10 300 python bench.py --workload c5-quota --no-cpu-baseline --steps 1 --warmup 0 > $o/qp.log 2>&1 || exit $?
