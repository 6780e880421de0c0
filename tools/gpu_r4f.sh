#!/bin/bash
# Round 4 measurement at a commit: the mask / bitmap parity tests, the default
# bench line (CPU baseline included, wall time recorded), then the three
# rocprofv3 passes of the C4 bench (tools/profile_box.sh).
set -o pipefail
T=${1:-r4f}
O=gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "mask or bitmap or row_list or frontier or pair_rows" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
s=$(date +%s)
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.log || { echo BENCH_FAILED; tail -30 $O/bench.log; exit 1; }
echo "bench wall $(( $(date +%s) - s )) s"
python -c "
import json; j=json.load(open('$O/bench.json')); r=j['roofline']; c=j['cpu_baseline']
print(j['ms_per_step'], j['value'], r['frac'], r.get('step_traffic_GBps'), j['dense_ms_per_step'])
print([round(x['avg_ms'],4) for x in j['frontier']['masked_sequence_ms']])
print({k: c[k] for k in c if k in ('value','unit','cores','kind')}, c.get('sample','')[:300])
print('dropin', {k: (j.get('dropin_module_step') or {}).get(k) for k in ('step_ms','forward_ms','adam_ms')})"
timeout -k 10 1000 bash tools/profile_box.sh $T > $O/profile.log 2>&1 || { echo PROFILE_FAILED; tail -30 $O/profile.log; exit 1; }
echo ALL_OK
