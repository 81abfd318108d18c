#!/bin/bash
# Timing variants of libfm_hip.so for tools/kbench.py A/B runs (never shipped):
#   tools/build_variant.sh <name> "<extra hipcc flags>" source.hip [source.hip ...]
# Reuses the in-tree objects and recompiles only the listed sources with the extra flags
# into build_variants/<name>/libfm_hip.so.
set -e
name=$1; flags=$2; shift 2
# the flags only reach the sources named here: with none the "variant" would be a copy
[ $# -ge 1 ] || { echo "build_variant: name the source(s) to rebuild with \"$flags\"" >&2; exit 2; }
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/fm-returnprediction_amd/csrc
VD=$ROOT/build_variants/$name
mkdir -p "$VD/obj"
cp -p "$CS"/build/*.o "$VD/obj/"
pids=()
for src in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I"$ROOT/include" \
    -Wall -Wno-unused-function $flags -c "$CS/$src" -o "$VD/obj/${src%.hip}.o" &
  pids+=($!)
done
for p in "${pids[@]}"; do
  wait "$p" || { echo "build_variant: a compile failed" >&2; rm -rf "$VD"; exit 1; }
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$VD"/obj/*.o -o "$VD/libfm_hip.so"
rm -rf "$VD/obj"
echo "$VD/libfm_hip.so"
