#!/bin/bash
# Round 4: small-graph chunk size sweep (C1 plain / v2_pop, C2) under graph
# replay, and one C1 kernel timeline.
set -o pipefail
O=gpurun_out/${1:-r4u}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 python3 -u tools/probes/chunk_probe.py --config C1 --variant plain --graph --steps 300 --chunks 2048,512,256,128,64 --thresholds 64,32 > $O/c1_plain.jsonl 2> $O/c1_plain.log || { tail -20 $O/c1_plain.log; exit 1; }
cat $O/c1_plain.jsonl
timeout -k 10 240 python3 -u tools/probes/chunk_probe.py --config C2 --graph --steps 200 --chunks 2048,512,256,128 --thresholds 64,32 > $O/c2.jsonl 2> $O/c2.log || { tail -20 $O/c2.log; exit 1; }
cat $O/c2.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace -T --output-format csv -d $O/trace_c1 -o run -- python3 bench.py --config C1 --variant plain --steps 20 --warmup 3 --no-cpu-baseline --no-torch-reference --dense-check 0 > $O/c1.json 2> $O/c1.log || { tail -20 $O/c1.log; exit 1; }
f=$(ls $O/trace_c1/*kernel_trace.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$(find $O/trace_c1 -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" --steps 4 > $O/c1_timeline.txt && head -60 $O/c1_timeline.txt
echo ALL_DONE
