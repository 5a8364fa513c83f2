#!/bin/bash
# Build libmxp from a git revision into ablib/libmxp_<name>.so (A/B against the working tree's build).
#   tools/mkablib_rev.sh <name> <rev>
set -eu
cd "$(dirname "$0")/.."
name=$1; rev=$2
t=$(mktemp -d /tmp/ablib.XXXXXX)
mkdir -p ablib
git archive "$rev" istio_amd/csrc istio_amd/build.py istio_amd/__init__.py include | tar -x -C "$t"
(cd "$t" && python -c "import sys; sys.path.insert(0,'.'); from istio_amd import build; build.build(force=True)" > "$t/build.log" 2>&1) || { cat "$t/build.log"; exit 1; }
cp "$t/istio_amd/libmxp.so" "ablib/libmxp_$name.so"
rm -rf "$t"
echo "ablib/libmxp_$name.so"
