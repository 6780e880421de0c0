# Round-end style check on the GPU box: the GPU test suite, smoke(), the
# default bench line, and a 2-rank rehearsal of the multi-GPU bench path over
# gloo (two ranks share the one GPU; RCCL needs one GPU per rank).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.log || { echo BENCH1_FAILED; tail -20 gpurun_out/bench1.log; exit 1; }
BBGR_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench2.json 2> gpurun_out/bench2.log || { echo BENCH2_FAILED; tail -30 gpurun_out/bench2.log; exit 1; }
python -c "
import json
for f in ('gpurun_out/bench1.json', 'gpurun_out/bench2.json'):
    j = json.load(open(f)); print(f, j['n_gpus'], round(j['ms_per_step'], 2), j['value'], j['scaling'])"
echo ALL_OK
