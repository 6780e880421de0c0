#!/bin/bash
# C2 (1M edges) single-GPU step, graph-replayed and eager, and the C4 line.
set -o pipefail
mkdir -p gpurun_out
T=${1:-c2}
timeout -k 10 200 python bench.py --config C2 --steps 300 --warmup 20 --no-cpu-baseline --dense-check 0 > gpurun_out/${T}_c2_graph.json 2> gpurun_out/${T}_c2_graph.log || { echo C2G_FAILED; tail -20 gpurun_out/${T}_c2_graph.log; exit 1; }
timeout -k 10 200 python bench.py --config C2 --steps 300 --warmup 20 --no-cpu-baseline --dense-check 0 --graph off > gpurun_out/${T}_c2_eager.json 2> gpurun_out/${T}_c2_eager.log || { echo C2E_FAILED; tail -20 gpurun_out/${T}_c2_eager.log; exit 1; }
timeout -k 10 200 python bench.py --config C1 --steps 300 --warmup 20 --no-cpu-baseline --dense-check 0 > gpurun_out/${T}_c1_graph.json 2> gpurun_out/${T}_c1_graph.log || { echo C1_FAILED; tail -20 gpurun_out/${T}_c1_graph.log; exit 1; }
echo ALL_OK
