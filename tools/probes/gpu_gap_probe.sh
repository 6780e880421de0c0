#!/bin/bash
# Inter-kernel gaps of the C4 fused step: eager vs graph replay, each under a
# rocprofv3 kernel trace (tools/step_timeline.py), plus the quick lines.
set -o pipefail
O=gpurun_out/$1; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
q="--steps 10 --warmup 2 --no-cpu-baseline --no-torch-reference --dense-check 0"
for g in off on; do
  timeout -k 10 300 python -u bench.py $q --graph $g > "$O/q_$g.json" 2> "$O/q_$g.log" || exit 1
  echo "graph $g: $(python tools/bench_brief.py "$O/q_$g.json" | head -1)"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tr_$g" -o run \
    -- python3 bench.py $q --graph $g --steps 5 > "$O/tr_$g.json" 2> "$O/tr_$g.log" || exit 1
  tr=$(find "$O/tr_$g" -name "*kernel_trace.csv" | head -1)
  python tools/step_timeline.py "$tr" --marker sample_kernel > "$O/timeline_$g.txt"
  sed -n '/median/p' "$O/timeline_$g.txt"
done
