set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench1.json 2> gpurun_out/bench1.log || { echo BENCH1_FAILED; exit 1; }
BBGR_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench2.json 2> gpurun_out/bench2.log || { echo BENCH2_FAILED; tail -30 gpurun_out/bench2.log; exit 1; }
echo ALL_OK
