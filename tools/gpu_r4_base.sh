#!/bin/bash
# Round-4 check on one GPU box: the GPU suite, smoke(), the N=8 user-row rank
# probe (+ a kernel trace of it) and the default bench line. A plain test
# failure (exit 1) does not stop the later steps; a fault, abort, segfault or
# time limit (exit 124 / 134 / 137 / 139) ends the script there.
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
hard() { case $1 in 124|134|137|139) echo "HARD FAIL ($1) in $2"; tail -30 "$3"; exit 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --durations=15 --timeout 500 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; hard $rc tests $O/gpu_tests.log
echo "TESTS rc=$rc"; grep -E "passed|failed" $O/gpu_tests.log | tail -2
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; hard $rc smoke $O/smoke.log; echo "SMOKE rc=$rc"; tail -1 $O/smoke.log
timeout -k 10 300 python -u tools/shard_probe.py --exchange-parts 1 --column-chains 1,2 --frontier-parts 1 > $O/shard8.jsonl 2> $O/shard8.log
rc=$?; hard $rc shard $O/shard8.log; echo "SHARD rc=$rc"; cat $O/shard8.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/shard8_trace -o run -- python3 tools/shard_probe.py --exchange-parts 1 --column-chains 1 --frontier-parts 1 --steps 10 > $O/shard8_trace.jsonl 2> $O/shard8_trace.log
rc=$?; hard $rc shardtrace $O/shard8_trace.log; echo "SHARDTRACE rc=$rc"
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.log
rc=$?; hard $rc bench $O/bench.log; echo "BENCH rc=$rc"
python -c "import json; j=json.load(open('$O/bench.json')); print(j['ms_per_step'], j['value'], j['roofline']['frac'], j['cpu_baseline']['sample'][:300])"
echo ALL_DONE
