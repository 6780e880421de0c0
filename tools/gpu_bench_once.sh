set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r30_bench.json 2> gpurun_out/r30_bench.log || { echo BENCH_FAILED; tail -30 gpurun_out/r30_bench.log; exit 1; }
python -c "
import json;j=json.load(open('gpurun_out/r30_bench.json'))
print(j['ms_per_step'], j['value'], j['roofline']['frac'])
print('torch', {k:v for k,v in j['torch_gpu_reference'].items() if k!='note'})
print('dropin', {k:v for k,v in j['dropin_module_step'].items() if k!='note'})
print('cpu', j['cpu_baseline']['value'], j['cpu_baseline']['step_s'])"
timeout -k 10 300 python bench.py --vertex-order input --no-cpu-baseline --no-torch-reference --dense-check 0 > gpurun_out/r30_bench_input.json 2> gpurun_out/r30_bench_input.log || { echo BENCH2_FAILED; tail -30 gpurun_out/r30_bench_input.log; exit 1; }
python -c "
import json;j=json.load(open('gpurun_out/r30_bench_input.json'))
print('input order', j['ms_per_step'])"
