set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3qp; mkdir -p $o
MXP_QUOTA_PROF=$o/prof.txt timeout -k 10 300 python bench.py --workload c5-quota --no-cpu-baseline --steps 1 --warmup 0 > $o/qp.log 2>&1 || exit $?
