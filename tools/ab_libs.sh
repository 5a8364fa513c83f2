#!/bin/bash
# Same-box A/B of two builds of libmxp (processes alternated, both orders): ab_libs.sh <workload> <libA> <libB> [env]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
wl=$1; a=$2; b=$3; shift 3
for lib in "$a" "$b" "$b" "$a"; do
    echo "== $lib"
    env "$@" MXP_LIB="$lib" timeout -k 10 200 python tools/ab.py "$wl" "" || exit $?
done
