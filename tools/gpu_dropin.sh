#!/bin/bash
# Drop-in module step (reference API + torch Adam) at C4: ops tests, then the
# probe with foreach and fused torch Adam, then a kernel-trace profile of it.
set -o pipefail
mkdir -p gpurun_out
T=${1:-dropin}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 300 python tools/dropin_probe.py --adam foreach > gpurun_out/${T}_foreach.json 2> gpurun_out/${T}_foreach.log || { echo FAIL1; tail -20 gpurun_out/${T}_foreach.log; exit 1; }
cat gpurun_out/${T}_foreach.json
timeout -k 10 300 python tools/dropin_probe.py --adam fused > gpurun_out/${T}_fused.json 2> gpurun_out/${T}_fused.log || { echo FAIL2; tail -20 gpurun_out/${T}_fused.log; exit 1; }
cat gpurun_out/${T}_fused.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o dropin -- python3 tools/dropin_probe.py --steps 5 --warmup 2 > gpurun_out/${T}_prof.log 2>&1 || { echo FAIL3; tail -20 gpurun_out/${T}_prof.log; exit 1; }
echo OK
