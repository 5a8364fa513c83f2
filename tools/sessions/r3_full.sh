# full GPU suite + smoke + secondary workloads at HEAD
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3full; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
for w in c3-ip c3-str c3-regex c5-quota; do
  timeout -k 10 300 python bench.py --workload $w > $o/bench_$w.log 2>&1 || exit $?
done
