set -o pipefail
mkdir -p gpurun_out/r11
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests/test_gpu_distributed.py -x -q > gpurun_out/r11/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r11/tests.log; exit 1; }
echo tests ok
timeout -k 10 300 python bench.py --sharded --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r11/sharded1.json 2> gpurun_out/r11/sharded1.log || { echo SH1_FAILED; tail -30 gpurun_out/r11/sharded1.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r11/trace -o run -- python3 bench.py --sharded --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r11/trace.json 2> gpurun_out/r11/trace.log || { echo PROF_FAILED; exit 1; }
echo ALL_OK
