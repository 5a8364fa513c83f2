#!/bin/bash
# Build an A/B variant of libmxp into ablib/libmxp_<name>.so from the working tree's sources with
# compile-time defaults of kernels.hip replaced: each NAME=VALUE rewrites `#define NAME ...`.
#   tools/mkablib_def.sh <name> NAME=VALUE [NAME=VALUE ...]
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
t=$(mktemp -d /tmp/ablib.XXXXXX)
mkdir -p "$t/istio_amd" ablib
cp -r istio_amd/csrc istio_amd/build.py istio_amd/__init__.py "$t/istio_amd/"
cp -r include "$t/"
for kv in "$@"; do
  k=${kv%%=*}; v=${kv#*=}
  grep -q "^#define $k " "$t/istio_amd/csrc/kernels.hip" || { echo "no #define $k"; exit 1; }
  sed -i "s/^#define $k .*/#define $k $v/" "$t/istio_amd/csrc/kernels.hip"
done
(cd "$t" && python -c "import sys; sys.path.insert(0,'.'); from istio_amd import build; build.build(force=True)" > "$t/build.log" 2>&1) || { cat "$t/build.log"; exit 1; }
cp "$t/istio_amd/libmxp.so" "ablib/libmxp_$name.so"
rm -rf "$t"
echo "ablib/libmxp_$name.so"
