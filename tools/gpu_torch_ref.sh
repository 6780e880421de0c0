#!/bin/bash
# Stock PyTorch-ROCm reference step (tools/torch_sparse_step.py) at C2 and C4.
set -o pipefail
mkdir -p gpurun_out
T=${1:-torchref}
for C in C2 C4; do
  timeout -k 10 400 python tools/torch_sparse_step.py --config $C > gpurun_out/${T}_$C.json 2> gpurun_out/${T}_$C.log || { echo FAIL $C; tail -20 gpurun_out/${T}_$C.log; exit 1; }
  cat gpurun_out/${T}_$C.json
done
echo OK
