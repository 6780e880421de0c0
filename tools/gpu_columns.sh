#!/bin/bash
# Column (embedding-dimension) sharding on the GPU box: parity tests, the
# per-rank step of N = 2, 4, 8 column shards on the C4 graph (one shard run
# alone on the one GPU), and a 2-rank gloo rehearsal of the column-sharded
# bench line.
set -o pipefail
mkdir -p gpurun_out
T=${1:-cols}
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -m gpu -x -q --timeout 300 --timeout-method thread -k "narrow or column or spmm_modes" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for n in 2 4 8; do
  timeout -k 10 300 python bench.py --emulate-columns $n --steps 20 --warmup 3 --no-cpu-baseline --dense-check 0 > gpurun_out/${T}_emul$n.json 2> gpurun_out/${T}_emul$n.log || { echo EMUL${n}_FAILED; tail -20 gpurun_out/${T}_emul$n.log; exit 1; }
done
BBGR_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --dense-check 0 > gpurun_out/${T}_gloo2.json 2> gpurun_out/${T}_gloo2.log || { echo GLOO2_FAILED; tail -30 gpurun_out/${T}_gloo2.log; exit 1; }
echo ALL_OK
