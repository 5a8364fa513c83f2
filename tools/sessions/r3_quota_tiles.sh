set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3qt; mkdir -p $o
for v in 512_2048 512_1024 512_512 1024_2048; do
  MXP_LIB=ablib/libmxp_q$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_memquota.py -x -q --timeout 200 --timeout-method thread > $o/t_$v.log 2>&1 || exit $?
done
for rep in 1 2; do
for v in 2048_2048 512_2048 512_1024 512_512 1024_2048; do
  echo "== $v" >> $o/q.log
  MXP_LIB=ablib/libmxp_q$v.so timeout -k 10 200 python bench.py --workload c5-quota --no-cpu-baseline --steps 20 --warmup 5 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernel_ms'])" >> $o/q.log || exit $?
done
done
