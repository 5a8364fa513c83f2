# round 6, session 14: regex dispatch stage ablations (stop after the probe / the header)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s14; mkdir -p $o
timeout -k 10 200 python -u tools/ab_rxp.py > $o/ab_rxp.log 2>&1 || exit $?
exit 0
