#!/bin/bash
# Round 4: A/B of the live-edge compaction in the masked SpMM gathers (in-tree
# build vs the previous spmm.hip and vs no occupancy target), then the N=8
# user-row rank probe at this commit.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=beyond-binary-fake-user-detection-a-credibility-aware-graph-based-recommender-system_amd
BENCH_ARGS="--no-torch-reference --dense-check 0" timeout -k 10 900 bash tools/probes/ab_spmm.sh $P/lib/ab/base/libbbgr.so $P/lib/ab/nowave/libbbgr.so || exit 1
python - <<'PY'
import json
for t in ("base", "v1", "v2"):
    j = json.load(open(f"gpurun_out/ab/{t}.json"))
    m = [round(x["avg_ms"], 4) for x in j["frontier"]["masked_sequence_ms"]]
    print(t, "(base=in-tree new, v1=old spmm, v2=new no wave target)", round(j["ms_per_step"], 3), m)
PY
mkdir -p gpurun_out/r4d
timeout -k 10 300 python -u tools/shard_probe.py --exchange-parts 1 --column-chains 1,2 --frontier-parts 1 > gpurun_out/r4d/shard8.jsonl 2> gpurun_out/r4d/shard8.log || { tail -20 gpurun_out/r4d/shard8.log; exit 1; }
cat gpurun_out/r4d/shard8.jsonl
echo ALL_OK
