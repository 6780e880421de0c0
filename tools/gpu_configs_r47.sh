#!/bin/bash
# BASELINE configs other than the default C4 line, at the final commit.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r47}
timeout -k 10 300 python bench.py --config C1 --steps 200 --warmup 20 --no-torch-reference > gpurun_out/${T}_c1.json 2> gpurun_out/${T}_c1.log || { echo C1_FAILED; tail -20 gpurun_out/${T}_c1.log; exit 1; }
timeout -k 10 400 python bench.py --config C3 --variant cu_fair --steps 20 --warmup 3 --no-cpu-baseline --no-torch-reference > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.log || { echo C3_FAILED; tail -20 gpurun_out/${T}_c3.log; exit 1; }
timeout -k 10 900 python bench.py --config C5 --steps 5 --warmup 1 --no-cpu-baseline --no-torch-reference > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.log || { echo C5_FAILED; tail -20 gpurun_out/${T}_c5.log; exit 1; }
for c in c1 c3 c5; do python -c "
import json; j=json.load(open('gpurun_out/${T}_$c.json')); print('$c', round(j['ms_per_step'],3), j['roofline']['frac'], j['config']['workload'])"; done
echo ALL_OK
