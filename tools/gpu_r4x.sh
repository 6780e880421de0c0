#!/bin/bash
# Round 4 late check at HEAD: the whole GPU suite, smoke(), the default bench
# line, then the three rocprofv3 passes of the C4 bench (tools/profile_box.sh).
set -o pipefail
T=${1:-r4x}
O=gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
hard() { case $1 in 124|134|137|139) echo "HARD FAIL ($1) in $2"; tail -30 "$3"; exit 1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --durations=10 --timeout 500 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; hard $rc tests $O/gpu_tests.log
echo "TESTS rc=$rc"; grep -E "passed|failed" $O/gpu_tests.log | tail -1; grep FAILED $O/gpu_tests.log | head
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; hard $rc smoke $O/smoke.log; echo "SMOKE rc=$rc"; tail -1 $O/smoke.log
[ $rc -eq 0 ] || exit 1
s=$(date +%s)
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.log
rc=$?; hard $rc bench $O/bench.log; echo "BENCH rc=$rc wall $(( $(date +%s) - s )) s"
[ $rc -eq 0 ] || exit 1
python -c "
import json; j=json.load(open('$O/bench.json')); r=j['roofline']; c=j['cpu_baseline']; dr=j['dropin_module_step']
print(j['ms_per_step'], j['value'], r['frac'], r.get('step_traffic_GBps'), j['dense_ms_per_step'])
print([round(x['avg_ms'],4) for x in j['frontier']['masked_sequence_ms']])
print('cpu', c['value'], c['cores'], c['sample'][:200]); print('dropin', {k: dr.get(k) for k in ('step_ms','forward_ms','forward_backward_ms','adam_ms')})"
timeout -k 10 1000 bash tools/profile_box.sh $T > $O/profile.log 2>&1 || { echo PROFILE_FAILED; tail -30 $O/profile.log; exit 1; }
echo ALL_DONE
