set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash tools/prof_session.sh r3v14/prof --no-c5 > gpurun_out/r3v14_prof.log 2>&1 || exit $?
