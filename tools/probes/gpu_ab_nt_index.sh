set -o pipefail
P=beyond-binary-fake-user-detection-a-credibility-aware-graph-based-recommender-system_amd
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BENCH_ARGS="--no-torch-reference --dense-check 0" timeout -k 10 1000 bash tools/probes/ab_spmm.sh $P/lib/ab/ntoff/libbbgr.so $P/lib/libbbgr.so $P/lib/ab/ntoff/libbbgr.so || exit 1
python - <<'PY'
import json
for t in ("base", "v1", "v2", "v3"):
    j = json.load(open(f"gpurun_out/ab/{t}.json")); f = j["frontier"]
    print(t, round(j["ms_per_step"], 3), [round(x["avg_ms"], 3) for x in f["full_sequence_ms"]], [round(x["avg_ms"], 3) for x in f["adam_sequence_ms"]], [round(x["avg_ms"], 3) for x in f["masked_sequence_ms"]])
PY
