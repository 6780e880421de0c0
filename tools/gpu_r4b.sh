#!/bin/bash
# Round-4 second check: the GPU test files the first check did not reach,
# the default bench line, and a host profile of the N=8 user-row rank.
set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
hard() { case $1 in 124|134|137|139) echo "HARD FAIL ($1) in $2"; tail -30 "$3"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_order.py tests/test_gpu_parity.py tests/test_gpu_distributed.py tests/test_gpu_graph.py -m gpu -v --durations=10 --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; hard $rc tests $O/gpu_tests.log
echo "TESTS rc=$rc"; grep -E "passed|failed" $O/gpu_tests.log | tail -2; grep FAILED $O/gpu_tests.log | head
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.log
rc=$?; hard $rc bench $O/bench.log; echo "BENCH rc=$rc"
python -c "import json; j=json.load(open('$O/bench.json')); print(j['ms_per_step'], j['value'], j['roofline']['frac'], j['roofline'].get('step_traffic_GBps'), j['cpu_baseline']['sample'][:400])" || tail -20 $O/bench.log
timeout -k 10 300 python -u tools/shard_probe.py --exchange-parts 1 --column-chains 1,2 --frontier-parts 1 --profile $O/shard8.prof > $O/shard8.jsonl 2> $O/shard8.log
rc=$?; hard $rc shard $O/shard8.log; echo "SHARD rc=$rc"; cat $O/shard8.jsonl
python - <<'PY'
import pstats, glob
for f in sorted(glob.glob("gpurun_out/r4b/shard8.prof.*")):
    print("==", f)
    pstats.Stats(f).sort_stats("tottime").print_stats(25)
PY
echo ALL_DONE
