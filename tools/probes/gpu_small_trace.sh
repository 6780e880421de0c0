#!/bin/bash
# Kernel timelines of the small configs' replayed steps (C2, C1).
set -o pipefail
O=gpurun_out/$1; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
q="--steps 30 --warmup 5 --no-cpu-baseline --no-torch-reference --dense-check 0"
for c in ${CONFIGS:-C2 C1}; do
  extra=""; [ $c = C1 ] && extra="--variant plain"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tr_$c" -o run \
    -- python3 bench.py --config $c $extra $q > "$O/tr_$c.json" 2> "$O/tr_$c.log" || exit 1
  tr=$(find "$O/tr_$c" -name "*kernel_trace.csv" | head -1)
  python tools/step_timeline.py "$tr" --marker sample_kernel > "$O/timeline_$c.txt"
  echo "$c: $(python tools/bench_brief.py "$O/tr_$c.json" | head -1)"; sed -n '/median/p' "$O/timeline_$c.txt"
done
