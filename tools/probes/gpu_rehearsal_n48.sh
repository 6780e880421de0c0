#!/bin/bash
# The driver's N=4 and N=8 bench commands rehearsed on a 1-GPU box: the ranks
# share cuda:0 over gloo (RCCL needs one GPU per rank), C4 strong scaling with
# the auto partition (columns at N=4, user rows at N=8). Correctness of the
# whole N>1 path, not its speed.
set -o pipefail
mkdir -p gpurun_out
T=${1:-rehearsal}
for N in ${NS:-4 8}; do
  BBGR_DIST_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 540 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2954$N bench.py --gpus $N --steps 2 --warmup 1 --dense-check 0 --weak-beside 1 --count-steps 1 --roofline-steps 1 > gpurun_out/${T}_gloo$N.json 2> gpurun_out/${T}_gloo$N.log || { echo GLOO${N}_FAILED; tail -30 gpurun_out/${T}_gloo$N.log; exit 1; }
  python -c "
import json;j=json.load(open('gpurun_out/${T}_gloo$N.json'))
print($N, j['partition'], j['config']['parallelism'], round(j['ms_per_step'],1), j['value'], j['config']['num_edges'], (j.get('weak_beside') or {}).get('num_edges'))"
done
echo ALL_OK
