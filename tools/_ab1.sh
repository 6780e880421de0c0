set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_order.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/ab/tests.log; exit 1; }
tail -1 gpurun_out/ab/tests.log
bash tools/gpu_measure.sh r3d dropin
