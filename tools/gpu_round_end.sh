#!/bin/bash
# Round-end record at the final commit: the full GPU test suite, then
# tools/gpu_final.sh (smoke, default bench twice, C2, drop-in, rocprofv3 passes).
set -o pipefail
mkdir -p gpurun_out
T=${1:-final}
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
bash tools/gpu_final.sh $T
