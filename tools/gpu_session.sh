#!/bin/bash
# One gpurun session: each GPU step under its own time limit; stop at the first crash / timeout
# (exit status >= 2 that is not a plain test failure).  Logs go to gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 limit=$2
    shift 2
    echo "== $name (limit ${limit}s): $*"
    timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 5 "gpurun_out/$name.log"
    if [ $rc -ge 2 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
    return 0
}
for s in "$@"; do
    eval "$s" || exit $?
done
