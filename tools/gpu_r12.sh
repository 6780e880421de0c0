#!/bin/bash
# Round-2 check: GPU tests (graph capture, in-launch split rows), C4 and C2
# bench lines (C2 graph-replayed and eager), C2 chunk-size probe.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r12}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || { echo BENCH_FAILED; tail -20 gpurun_out/${T}_bench.log; exit 1; }
timeout -k 10 200 python bench.py --config C2 --steps 300 --warmup 20 --no-cpu-baseline --dense-check 0 > gpurun_out/${T}_c2_graph.json 2> gpurun_out/${T}_c2_graph.log || { echo C2G_FAILED; tail -20 gpurun_out/${T}_c2_graph.log; exit 1; }
timeout -k 10 200 python bench.py --config C2 --steps 300 --warmup 20 --no-cpu-baseline --dense-check 0 --graph off > gpurun_out/${T}_c2_eager.json 2> gpurun_out/${T}_c2_eager.log || { echo C2E_FAILED; tail -20 gpurun_out/${T}_c2_eager.log; exit 1; }
timeout -k 10 200 python tools/chunk_probe.py --config C2 > gpurun_out/${T}_chunk_probe.jsonl 2> gpurun_out/${T}_chunk_probe.log || { echo PROBE_FAILED; tail -20 gpurun_out/${T}_chunk_probe.log; exit 1; }
echo ALL_OK
