#!/bin/bash
# Round 4: the GPU suite (stop at the first failure), the N=8 rank probe with
# torch's collectives and with every collective inline on the compute stream,
# and the C4 bench line (no CPU / stock-torch legs).
set -o pipefail
O=gpurun_out/${1:-r4j}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
hard() { case $1 in 124|134|137|139) echo "HARD FAIL ($1) in $2"; tail -30 "$3"; exit 1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --durations=10 --timeout 500 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; hard $rc tests $O/gpu_tests.log
echo "TESTS rc=$rc"; grep -E "passed|failed" $O/gpu_tests.log | tail -2; grep FAILED $O/gpu_tests.log | head -20
[ $rc -eq 0 ] || exit 1
for nc in off inline; do
timeout -k 10 300 python -u tools/shard_probe.py --exchange-parts 1 --column-chains 1 --frontier-parts 1 --native-comm $nc > $O/shard8_$nc.jsonl 2> $O/shard8_$nc.log
rc=$?; hard $rc shard $O/shard8_$nc.log; [ $rc -eq 0 ] || { tail -20 $O/shard8_$nc.log; exit 1; }
grep config $O/shard8_$nc.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace -T --output-format csv -d $O/trace -o run -- python3 tools/shard_probe.py --exchange-parts 1 --column-chains 1 --frontier-parts 1 --native-comm inline --steps 10 > $O/trace.jsonl 2> $O/trace.log || { tail -20 $O/trace.log; exit 1; }
python tools/step_timeline.py $(find $O/trace -name "*kernel_trace.csv" | head -1) --steps 6 > $O/timeline.txt && head -9 $O/timeline.txt
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-torch-reference --dense-check 0 > $O/bench.json 2> $O/bench.log
rc=$?; hard $rc bench $O/bench.log; echo "BENCH rc=$rc"
python -c "
import json; j=json.load(open('$O/bench.json')); f=j['frontier']
print(j['ms_per_step'], j['value'], j['roofline']['frac'])"
echo ALL_DONE
