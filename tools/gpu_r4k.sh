#!/bin/bash
# Round 4: kernel traces of the small-graph steps (C1 plain, C2), cut into steps.
set -o pipefail
O=gpurun_out/r4k
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in "C1 --variant plain" "C2"; do
  t=$(echo $c | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --kernel-trace -T --output-format csv -d $O/trace_$t -o run -- python3 bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-torch-reference --dense-check 0 > $O/$t.json 2> $O/$t.log || { tail -20 $O/$t.log; exit 1; }
  python tools/step_timeline.py $(find $O/trace_$t -name "*kernel_trace.csv" | head -1) --steps 8 > $O/timeline_$t.txt; head -12 $O/timeline_$t.txt
done
echo ALL_OK
