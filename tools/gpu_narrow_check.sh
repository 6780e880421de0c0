#!/bin/bash
# Narrow-kernel settings: parity tests that run narrow widths, then one column
# shard of 2 and of 4, and the default C4 line.
set -o pipefail
mkdir -p gpurun_out/abn
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -m gpu -x -q --timeout 300 --timeout-method thread -k "narrow or column or spmm_modes or chains or fused_adam" > gpurun_out/abn/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/abn/tests.log; exit 1; }
tail -1 gpurun_out/abn/tests.log
for P in 2 4; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-torch-reference --dense-check 0 --emulate-columns $P > gpurun_out/abn/new_c$P.json 2> gpurun_out/abn/new_c$P.log || { echo BENCH_FAILED; tail -20 gpurun_out/abn/new_c$P.log; exit 1; }
  python -c "
import json;j=json.load(open('gpurun_out/abn/new_c$P.json'))
print('cols$P', round(j['ms_per_step'],3), [(k['kind'],k['side'][:4],k.get('masks',''),round(k['avg_ms'],3)) for k in j['roofline']['per_kernel']])"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-torch-reference --dense-check 0 > gpurun_out/abn/new_c4.json 2> gpurun_out/abn/new_c4.log || { echo BENCH_FAILED; exit 1; }
python -c "
import json;j=json.load(open('gpurun_out/abn/new_c4.json')); print('C4', round(j['ms_per_step'],3), round(j['roofline']['frac'],4))"
