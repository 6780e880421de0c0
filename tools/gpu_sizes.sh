set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 600 python -m pytest tests/test_gpu_distributed.py tests/test_gpu_parity.py -x -q > gpurun_out/r4/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r4/tests.log; exit 1; }
echo tests ok
timeout -k 10 400 python bench.py --config C3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r4/c3.json 2> gpurun_out/r4/c3.log || { echo C3_FAILED; tail -20 gpurun_out/r4/c3.log; exit 1; }
echo c3 ok
timeout -k 10 900 python bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4/c5.json 2> gpurun_out/r4/c5.log || { echo C5_FAILED; tail -20 gpurun_out/r4/c5.log; exit 1; }
echo ALL_OK
