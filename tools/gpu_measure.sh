#!/bin/bash
# On the GPU box, from the repo root: the default bench line (C4 + CPU
# baseline), the C2 line, and the three rocprofv3 passes of tools/profile_box.sh.
# Usage: tools/gpu_measure.sh <tag>
set -o pipefail
TAG=${1:-rXX}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log \
  || { echo BENCH_FAILED; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
timeout -k 10 200 python bench.py --config C2 --steps 200 --warmup 20 --no-cpu-baseline \
  > gpurun_out/${TAG}_c2_bench.json 2> gpurun_out/${TAG}_c2_bench.log \
  || { echo C2_FAILED; tail -20 gpurun_out/${TAG}_c2_bench.log; exit 1; }
bash tools/profile_box.sh $TAG || { echo PROFILE_FAILED; exit 1; }
echo MEASURE_OK
