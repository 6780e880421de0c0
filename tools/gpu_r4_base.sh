#!/bin/bash
# Round-4 start: GPU suite + smoke + default bench at HEAD, then the N=8
# user-row rank probe with a kernel trace (per-kernel times of one rank).
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "FAIL $1"; tail -30 "$2"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --durations=15 --timeout 500 --timeout-method thread > $O/gpu_tests.log 2>&1 || fail tests $O/gpu_tests.log
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail smoke $O/smoke.log
tail -1 $O/smoke.log
timeout -k 10 300 python -u tools/shard_probe.py --exchange-parts 1 --column-chains 1,2 --frontier-parts 1 > $O/shard8.jsonl 2> $O/shard8.log || fail shard $O/shard8.log
cat $O/shard8.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/shard8_trace -o run -- python3 tools/shard_probe.py --exchange-parts 1 --column-chains 1 --frontier-parts 1 --steps 10 > $O/shard8_trace.jsonl 2> $O/shard8_trace.log || fail shardtrace $O/shard8_trace.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.log || fail bench $O/bench.log
python -c "import json; j=json.load(open('$O/bench.json')); print(j['ms_per_step'], j['value'], j['roofline']['frac'])"
echo ALL_OK
