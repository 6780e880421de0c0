set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_order.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/ab/tests.log; exit 1; }
tail -1 gpurun_out/ab/tests.log
SKIP_TESTS=1 bash tools/ab_spmm.sh beyond-binary-fake-user-detection-a-credibility-aware-graph-based-recommender-system_amd/lib/ab/rw8/libbbgr.so beyond-binary-fake-user-detection-a-credibility-aware-graph-based-recommender-system_amd/lib/ab/pw8/libbbgr.so beyond-binary-fake-user-detection-a-credibility-aware-graph-based-recommender-system_amd/lib/ab/both/libbbgr.so
