# round 4, session 2: Go strings.ToUpper lists (new GPU parity tests) + list and parity suites
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r4s2; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_lists.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $o/t.log 2>&1 || exit $?
