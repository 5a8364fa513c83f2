# round 6, session 10: where a fresh C2 step goes (kernel + memory-copy trace of the group's fresh
# loop, narrow wire), host call times of one step.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r6s10; mkdir -p $o
timeout -k 10 240 python -u tools/fresh_group_prof.py c2 8 narrow > $o/plain.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $o/prof -o fresh -- python3 -u tools/fresh_group_prof.py c2 8 narrow > $o/prof.log 2>&1 || exit $?
exit 0
