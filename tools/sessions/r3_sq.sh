set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash tools/sq_session.sh r3sq_c4 --workload c4 > gpurun_out/r3sq_c4.log 2>&1 || exit $?
