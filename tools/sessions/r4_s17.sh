# round 4, session 17: where a fresh-batch step's time goes -- the bench's fresh loop under
# rocprofv3 --hip-trace --kernel-trace --stats (HIP API calls: copies, allocations, frees, syncs)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MXP_NO_BUILD=1
o=gpurun_out/r4s17; mkdir -p $o
for w in c2 c4; do
    timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $o/fresh_$w -o run -- python3 tools/fresh_prof.py $w 6 > $o/fresh_$w.log 2>&1 || exit $?
done
