#!/bin/bash
# Round 3: drop-in module step with the degree-ordered drop-in graph (A/B
# against the input-order graph on the same box), then the default bench line.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r3}
for o in degree input; do
  BBGR_DROPIN_ORDER=$o timeout -k 10 300 python tools/dropin_probe.py --adam bbgr \
    > gpurun_out/${T}_dropin_bbgr_$o.json 2> gpurun_out/${T}_dropin_bbgr_$o.log || { echo FAIL_$o; tail -20 gpurun_out/${T}_dropin_bbgr_$o.log; exit 1; }
  cat gpurun_out/${T}_dropin_bbgr_$o.json
done
timeout -k 10 300 python tools/dropin_probe.py --adam foreach > gpurun_out/${T}_dropin_foreach.json 2> gpurun_out/${T}_dropin_foreach.log || { echo FAIL_foreach; exit 1; }
cat gpurun_out/${T}_dropin_foreach.json
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench1.json 2> gpurun_out/${T}_bench1.log || { echo FAIL_bench; tail -30 gpurun_out/${T}_bench1.log; exit 1; }
echo OK
