#!/bin/bash
# A/B: bench.py's HW-queue raise (GPU_MAX_HW_QUEUES 4 -> 8) against the box
# default, quick C4 lines and one kernel trace each (inter-kernel gaps).
set -o pipefail
O=gpurun_out/$1; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
q="--steps 10 --warmup 2 --no-cpu-baseline --no-torch-reference --dense-check 0"
for mode in keep raise keep raise; do
  if [ $mode = keep ]; then export BBGR_KEEP_HW_QUEUES=1; else unset BBGR_KEEP_HW_QUEUES; fi
  timeout -k 10 300 python -u bench.py $q > "$O/q_$mode.json" 2> "$O/q_$mode.log" || exit 1
  echo "$mode: $(python tools/bench_brief.py "$O/q_$mode.json" | head -1)"
done
for mode in keep raise; do
  if [ $mode = keep ]; then export BBGR_KEEP_HW_QUEUES=1; else unset BBGR_KEEP_HW_QUEUES; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tr_$mode" -o run \
    -- python3 bench.py $q --steps 5 > "$O/tr_$mode.json" 2> "$O/tr_$mode.log" || exit 1
  tr=$(find "$O/tr_$mode" -name "*kernel_trace.csv" | head -1)
  python tools/step_timeline.py "$tr" --marker sample_kernel > "$O/timeline_$mode.txt"
  echo "$mode trace: $(sed -n 2,12p "$O/timeline_$mode.txt" | grep -c .) steps"; sed -n '/median/p' "$O/timeline_$mode.txt"
done
