#!/bin/bash
# Build libcordahip with extra compile definitions into build_ab/<name>/libcordahip.so (A/B runs:
# CORDAHIP_LIB=build_ab/<name>/libcordahip.so).  Usage: tools/build_variant.sh <name> -DFOO=1 ...
set -euo pipefail
cd "$(dirname "$0")/.."
NAME=$1; shift
OUT=build_ab/$NAME
mkdir -p $OUT
objs=()
for f in runtime ed25519 ed25519_comb ecdsa txid uniq signers kryo group; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c corda_amd/csrc/$f.hip -o $OUT/$f.o -I include "$@" &
  objs+=($OUT/$f.o)
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libcordahip.so "${objs[@]}"
echo $OUT/libcordahip.so
