# round 5, session 19: the device CIDR list against Python ipaddress.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r5s19; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_ip_vs_python_ipaddress.py -m gpu -x -v --timeout 200 --timeout-method thread > $o/t.log 2>&1 || exit $?
