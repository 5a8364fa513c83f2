# round-5 closing build, repeat: the default bench line twice more on a fresh box (run-to-run spread
# of the C2 / C4 / C5 steps, the fresh-batch and end-to-end blocks).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5h2; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib.sha1
timeout -k 10 500 python -u bench.py > $o/bench1.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --no-cpu-baseline > $o/bench2.log 2>&1 || exit $?
