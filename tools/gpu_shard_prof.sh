#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/shardprof -o run -- python3 tools/shard_probe.py --parts-of 8 --exchange-parts 4 --steps 20 > gpurun_out/shardprof.log 2>&1 || { echo FAIL; tail -20 gpurun_out/shardprof.log; exit 1; }
find gpurun_out/shardprof -name "*kernel_stats.csv"
