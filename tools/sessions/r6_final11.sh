# round 6, final session 11: the final tree (kernels of fingerprint 567fca63, the ragged-batch and
# small-group tests added): the whole GPU suite, smoke, the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6k; mkdir -p $o
python3 -c "import bench; print(bench.kernel_fingerprint())" > $o/fingerprint.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > $o/bench.log 2>&1 || exit $?
exit 0
