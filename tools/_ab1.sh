set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_order.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/ab/tests.log; exit 1; }
tail -1 gpurun_out/ab/tests.log
timeout -k 10 300 python tools/dropin_ops_probe.py > gpurun_out/ab/dropin_ops.txt 2>&1 || { echo PROBE_FAILED; tail -30 gpurun_out/ab/dropin_ops.txt; exit 1; }
BBGR_DROPIN_ORDER=degree timeout -k 10 300 python tools/dropin_probe.py --adam bbgr > gpurun_out/ab/dropin_bbgr_degree.json 2> gpurun_out/ab/dropin.log || { echo DROPIN_FAILED; tail -20 gpurun_out/ab/dropin.log; exit 1; }
cat gpurun_out/ab/dropin_bbgr_degree.json
