# round 6, session 3: the whole GPU suite on the device-group build (group C-ABI, resolve over
# uploaded batches, pack_pending fix), then the default bench line through the group.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s3; mkdir -p $o
sha1sum istio_amd/libmxp.so > $o/lib.sha1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || exit $?
timeout -k 10 450 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $o/bench.log 2>&1 || exit $?
