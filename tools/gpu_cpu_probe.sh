#!/bin/bash
# CPU-baseline spread on the box host: 3 runs free-floating, 3 runs pinned to
# 16 CPUs of one NUMA node.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python tools/cpu_baseline_probe.py --runs 3 --pin 0 > gpurun_out/cpuprobe_free.jsonl 2> gpurun_out/cpuprobe_free.log || { echo FREE_FAILED; tail -20 gpurun_out/cpuprobe_free.log; exit 1; }
timeout -k 10 500 python tools/cpu_baseline_probe.py --runs 3 --pin 16 > gpurun_out/cpuprobe_pin.jsonl 2> gpurun_out/cpuprobe_pin.log || { echo PIN_FAILED; tail -20 gpurun_out/cpuprobe_pin.log; exit 1; }
python -c "
import json
for f in ('free','pin'):
    for l in open(f'gpurun_out/cpuprobe_{f}.jsonl'):
        j=json.loads(l); print(f, round(j['step_s'],2), {k:round(v,2) for k,v in j['components_s'].items()}, round(j['wall_s']))"
