#!/bin/bash
# Build an A/B variant of libbbgr.so with extra -D flags (tools/probes/ab_spmm.sh runs
# bench.py against it through BBGR_LIB). Only one source is rebuilt (SRC, default
# spmm); the other objects come from the in-tree build (run build() first).
# Usage: [SRC=eval] tools/probes/build_variant.sh <tag> -DFLAG=VALUE ...
set -euo pipefail
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
PKG=$(ls -d "$ROOT"/beyond-binary-*_amd)
OUT=$PKG/lib/ab/$TAG
mkdir -p "$OUT"
HIPCC=/opt/rocm/bin/hipcc
SRC=${SRC:-spmm}
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/include" -Wall -Wno-unused-function \
  "$@" -c "$PKG/csrc/$SRC.hip" -o "$OUT/$SRC.o"
OBJS="$OUT/$SRC.o"
for o in spmm graph train eval cred comm; do
  [ "$o" = "$SRC" ] || OBJS="$OBJS $PKG/lib/obj/$o.o"
done
$HIPCC --offload-arch=gfx950 -shared -fPIC -o "$OUT/libbbgr.so" $OBJS -ldl
echo "${OUT#$ROOT/}/libbbgr.so"
