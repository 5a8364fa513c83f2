# round 6, session 13: regex dispatch A/B with the tail classes from registers (MXP_LIST_OPT bit 16, since removed: no gain)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s13; mkdir -p $o
timeout -k 10 200 python -u tools/ab_rxp.py > $o/ab_rxp.log 2>&1 || exit $?
exit 0
