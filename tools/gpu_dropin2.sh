#!/bin/bash
# Drop-in module step at C4 after a change to the drop-in path: the ops tests,
# the probe with foreach torch Adam and with bbgr FusedAdam, and a kernel trace.
set -o pipefail
mkdir -p gpurun_out
T=${1:-dropin}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for A in foreach bbgr; do
  timeout -k 10 300 python tools/dropin_probe.py --adam $A > gpurun_out/${T}_$A.json 2> gpurun_out/${T}_$A.log || { echo FAIL_$A; tail -20 gpurun_out/${T}_$A.log; exit 1; }
  cat gpurun_out/${T}_$A.json
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o dropin -- python3 tools/dropin_probe.py --steps 5 --warmup 2 > gpurun_out/${T}_prof.log 2>&1 || { echo FAIL_PROF; tail -20 gpurun_out/${T}_prof.log; exit 1; }
echo OK
