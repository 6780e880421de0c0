#!/bin/bash
# A/B of the narrow (column-shard) kernels: one column shard of 2 (32 columns)
# and of 4 (16 columns) with the in-tree build and lib/ab variants
# (VARIANTS="tag:parts:libdir ..."; r32 runs: c2base/c2r1/c2w8/c2r1w8, c4base/c4r1).
set -o pipefail
mkdir -p gpurun_out/abn
L=beyond-binary-fake-user-detection-a-credibility-aware-graph-based-recommender-system_amd/lib/ab
run() {  # tag, parts, lib
  local tag=$1; local parts=$2; local lib=$3
  env ${lib:+BBGR_LIB=$PWD/$L/$lib/libbbgr.so} timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-torch-reference --dense-check 0 --emulate-columns $parts > gpurun_out/abn/$tag.json 2> gpurun_out/abn/$tag.log || { echo "BENCH $tag FAILED"; tail -20 gpurun_out/abn/$tag.log; exit 1; }
  python -c "
import json;j=json.load(open('gpurun_out/abn/$tag.json'))
print('$tag', round(j['ms_per_step'],3), [(k['kind'],k['side'][:4],k.get('masks',''),round(k['avg_ms'],3)) for k in j['roofline_per_kernel']])"
}
VARIANTS=${VARIANTS:-"c4base:4: c4w16:4:w16 c4mw16:4:mw16 c4r3:4:r3s16 c4base_b:4:"}
for v in $VARIANTS; do
  IFS=: read tag parts lib <<< "$v"
  run $tag $parts "$lib" || exit 1
done
echo ALL_OK
