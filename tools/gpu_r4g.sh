#!/bin/bash
# Round 4: the whole GPU suite at this commit, then the C4 bench without the
# CPU / stock-torch legs (step time and the per-launch sequences).
set -o pipefail
O=gpurun_out/${1:-r4g}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
hard() { case $1 in 124|134|137|139) echo "HARD FAIL ($1) in $2"; tail -30 "$3"; exit 1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --durations=10 --timeout 500 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; hard $rc tests $O/gpu_tests.log
echo "TESTS rc=$rc"; grep -E "passed|failed" $O/gpu_tests.log | tail -2; grep FAILED $O/gpu_tests.log | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-torch-reference --dense-check 0 > $O/bench.json 2> $O/bench.log
rc=$?; hard $rc bench $O/bench.log; echo "BENCH rc=$rc"
python -c "
import json; j=json.load(open('$O/bench.json')); f=j['frontier']
print(j['ms_per_step'], j['value'], j['roofline']['frac'])
for k in ('full_sequence_ms','adam_sequence_ms','masked_sequence_ms'): print(k, [round(x['avg_ms'],4) for x in f[k]])"
echo ALL_DONE
