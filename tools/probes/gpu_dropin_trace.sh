#!/bin/bash
# Round 4: kernel timeline of the drop-in step (deferred tables, FusedAdam).
set -o pipefail
O=gpurun_out/dropin_trace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -T --output-format csv -d $O/trace -o run -- python3 tools/dropin_probe.py --adam bbgr --steps 6 > $O/probe.json 2> $O/probe.log || { tail -20 $O/probe.log; exit 1; }
F=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python tools/step_timeline.py $F --marker bpr_reduce_kernel --steps 40 > $O/segments.txt || true
head -45 $O/segments.txt
# the timed step() calls follow 3 warm-up steps (one BPR forward each)
python tools/step_timeline.py $F --marker bpr_reduce_kernel --index 5 > $O/timeline.txt || true
sed -n 1,140p $O/timeline.txt
echo ALL_OK
