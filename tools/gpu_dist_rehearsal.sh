#!/bin/bash
# Multi-rank bench rehearsal on a 1-GPU box: 2 ranks over gloo sharing the
# GPU (strong scaling of C4, the N>1 default), and the sharded trainer at N=1
# over RCCL (its own overhead against the single-GPU step).
set -o pipefail
mkdir -p gpurun_out
T=${1:-rehearsal}
BBGR_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --dense-check 0 --weak-beside 2 > gpurun_out/${T}_gloo2.json 2> gpurun_out/${T}_gloo2.log || { echo GLOO2_FAILED; tail -30 gpurun_out/${T}_gloo2.log; exit 1; }
timeout -k 10 400 python bench.py --sharded --steps 20 --warmup 3 --no-cpu-baseline --dense-check 0 > gpurun_out/${T}_sharded1.json 2> gpurun_out/${T}_sharded1.log || { echo SHARDED1_FAILED; tail -30 gpurun_out/${T}_sharded1.log; exit 1; }
echo ALL_OK
