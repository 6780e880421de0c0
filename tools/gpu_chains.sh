#!/bin/bash
# Column chains (ShardedTrainer column_chains=2): distributed + graph GPU
# tests, then the sharded C4 step at N=1 over RCCL with 1 and 2 chains (the
# chains' compute overhead; the overlap they buy needs N > 1 links).
set -o pipefail
mkdir -p gpurun_out
T=${1:-chains}
timeout -k 10 900 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_graph.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for C in 1 2; do
  timeout -k 10 300 python bench.py --sharded --partition users --no-cpu-baseline --dense-check 0 --weak-beside 0 --column-chains $C > gpurun_out/${T}_c4_ch$C.json 2> gpurun_out/${T}_c4_ch$C.log || { echo BENCH_FAILED $C; tail -20 gpurun_out/${T}_c4_ch$C.log; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/${T}_c4_ch$C.json'));print($C, j['ms_per_step'], j['value'])"
done
echo ALL_OK
