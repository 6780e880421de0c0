#!/bin/bash
# Round 4: deferred drop-in tables — the lazy / ops / parity GPU tests, then
# the C4 drop-in step with deferred and with dense finals (FusedAdam, foreach).
set -o pipefail
O=gpurun_out/${1:-r4o}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_lazy.py tests/test_gpu_ops.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; tail -40 $O/tests.log; exit 1; }
for a in "--adam bbgr" "--adam bbgr --dense-finals" "--adam foreach"; do
  t=$(echo $a | tr -d ' -')
  timeout -k 10 300 python tools/dropin_probe.py $a > $O/dropin_$t.json 2> $O/dropin_$t.log || { tail -20 $O/dropin_$t.log; exit 1; }
  python -c "import json; j=json.load(open('$O/dropin_$t.json')); print('$a', {k: round(j[k],3) for k in ('step_ms','forward_ms','full_tables_ms','forward_backward_ms','adam_ms')}, j['lazy_finals'])"
done
echo ALL_OK
