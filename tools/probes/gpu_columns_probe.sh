#!/bin/bash
# Round 4: one embedding-column shard of C4 alone (bench.py --emulate-columns N:
# rank 0's d/N columns, whole graph) at N = 2, 4: step time and per-launch times.
set -o pipefail
O=gpurun_out/cols
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in 2 4; do
  timeout -k 10 300 python -u bench.py --emulate-columns $n --steps 10 --no-cpu-baseline --no-torch-reference --dense-check 0 > $O/cols$n.json 2> $O/cols$n.log || { tail -20 $O/cols$n.log; exit 1; }
  python -c "
import json; j=json.load(open('$O/cols$n.json')); f=j['frontier']
print($n, round(j['ms_per_step'],3), [round(x['avg_ms'],3) for x in f['full_sequence_ms']], [round(x['avg_ms'],3) for x in f['adam_sequence_ms']], [round(x['avg_ms'],3) for x in f['masked_sequence_ms']])"
done
timeout -k 10 300 rocprofv3 --kernel-trace -T --output-format csv -d $O/trace4 -o run -- python3 bench.py --emulate-columns 4 --steps 10 --no-cpu-baseline --no-torch-reference --dense-check 0 > $O/trace4.json 2> $O/trace4.log || { tail -20 $O/trace4.log; exit 1; }
python tools/step_timeline.py $(find $O/trace4 -name "*kernel_trace.csv" | head -1) --steps 16 > $O/timeline4.txt && sed -n 1,80p $O/timeline4.txt
echo ALL_OK
