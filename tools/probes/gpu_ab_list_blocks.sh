#!/bin/bash
# A/B: short-row workgroups of device-length row-list launches (BBGR_LIST_BLOCKS,
# the grid-stride cap) on the C4 bench: uncapped (the capacity grid) vs capped.
set -o pipefail
O=gpurun_out/${1:-ablist}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
for lb in 1000000000 8192 2048; do
  BBGR_LIST_BLOCKS=$lb timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-torch-reference --dense-check 0 > $O/lb${lb}_$rep.json 2> $O/lb${lb}_$rep.log || { tail -20 $O/lb${lb}_$rep.log; exit 1; }
  python3 -c "
import json; j=json.load(open('$O/lb${lb}_$rep.json')); m=j['frontier']['masked_sequence_ms']
print('$lb', round(j['ms_per_step'],3), [round(x['avg_ms'],4) for x in m])"
done; done
echo ALL_DONE
