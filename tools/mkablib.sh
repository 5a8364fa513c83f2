#!/bin/bash
# Build an A/B variant of libmxp into ablib/libmxp_<name>.so: the working tree's sources, plus an
# optional patch, compiled in a scratch copy (the in-tree library is untouched).
#   tools/mkablib.sh <name> [patch]
set -eu
cd "$(dirname "$0")/.."
name=$1; patch=${2:-}
t=$(mktemp -d /tmp/ablib.XXXXXX)
mkdir -p "$t/istio_amd" ablib
cp -r istio_amd/csrc istio_amd/build.py istio_amd/__init__.py "$t/istio_amd/"
cp -r include "$t/"
if [ -n "$patch" ]; then (cd "$t" && patch -p1 -s < "$OLDPWD/$patch"); fi
(cd "$t" && python -c "import sys; sys.path.insert(0,'.'); from istio_amd import build; build.build(force=True)" > "$t/build.log" 2>&1) || { cat "$t/build.log"; exit 1; }
cp "$t/istio_amd/libmxp.so" "ablib/libmxp_$name.so"
rm -rf "$t"
echo "ablib/libmxp_$name.so"
