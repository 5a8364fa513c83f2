# round 6, session 18: kernel times of the regex A/B (sort kernels vs the walk)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s18; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o ab -- python3 -u tools/ab_rxp.py > $o/ab_rxp.log 2>&1 || exit $?
exit 0
