#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/shard_probe.py --parts-of 8 --exchange-parts 1,2,4,8 > gpurun_out/shard8.jsonl 2> gpurun_out/shard8.log || { echo FAIL8; tail -20 gpurun_out/shard8.log; exit 1; }
cat gpurun_out/shard8.jsonl
timeout -k 10 400 python tools/shard_probe.py --parts-of 4 --exchange-parts 2,4,8 > gpurun_out/shard4.jsonl 2> gpurun_out/shard4.log || { echo FAIL4; tail -20 gpurun_out/shard4.log; exit 1; }
cat gpurun_out/shard4.jsonl
