#!/bin/bash
# A/B of the narrow (column-shard) kernels: one column shard of 2 (32 columns)
# and of 4 (16 columns) with the in-tree build and lib/ab variants.
set -o pipefail
mkdir -p gpurun_out/abn
L=beyond-binary-fake-user-detection-a-credibility-aware-graph-based-recommender-system_amd/lib/ab
run() {  # tag, parts, lib
  local tag=$1; local parts=$2; local lib=$3
  env ${lib:+BBGR_LIB=$PWD/$L/$lib/libbbgr.so} timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-torch-reference --dense-check 0 --emulate-columns $parts > gpurun_out/abn/$tag.json 2> gpurun_out/abn/$tag.log || { echo "BENCH $tag FAILED"; tail -20 gpurun_out/abn/$tag.log; exit 1; }
  python -c "
import json;j=json.load(open('gpurun_out/abn/$tag.json'))
print('$tag', round(j['ms_per_step'],3), [(k['kind'],k['side'][:4],k.get('masks',''),round(k['avg_ms'],3)) for k in j['roofline']['per_kernel']])"
}
run c2base 2 "" && run c2r1 2 r1 && run c2w8 2 w8 && run c2r1w8 2 r1w8 && run c2base_b 2 "" && \
run c4base 4 "" && run c4r1 4 r1s16 && echo ALL_OK
