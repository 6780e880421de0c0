#!/bin/bash
# Build an A/B variant of libbbgr.so with extra -D flags (tools/probes/ab_spmm.sh runs
# bench.py against it through BBGR_LIB). Only spmm.hip is rebuilt; the other
# objects come from the in-tree build (run build() first).
# Usage: tools/probes/build_variant.sh <tag> -DFLAG=VALUE ...
set -euo pipefail
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
PKG=$(ls -d "$ROOT"/beyond-binary-*_amd)
OUT=$PKG/lib/ab/$TAG
mkdir -p "$OUT"
HIPCC=/opt/rocm/bin/hipcc
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/include" -Wall -Wno-unused-function \
  "$@" -c "$PKG/csrc/spmm.hip" -o "$OUT/spmm.o"
OBJS="$OUT/spmm.o"
for o in graph train eval cred comm; do OBJS="$OBJS $PKG/lib/obj/$o.o"; done
$HIPCC --offload-arch=gfx950 -shared -fPIC -o "$OUT/libbbgr.so" $OBJS -ldl
echo "${OUT#$ROOT/}/libbbgr.so"
