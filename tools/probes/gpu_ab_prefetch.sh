#!/bin/bash
# A/B: fused-Adam kernels with the param/moment prefetch (in-tree build) vs
# without (lib/ab/nopf), C4 twice interleaved, C3 cu_fair once each.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/ab/tests.log; exit 1; }
tail -1 gpurun_out/ab/tests.log
run() {  # tag, args, env...
  local tag=$1; local args=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-torch-reference --dense-check 0 $args > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.log || { echo "BENCH $tag FAILED"; tail -20 gpurun_out/ab/$tag.log; exit 1; }
  python -c "
import json;j=json.load(open('gpurun_out/ab/$tag.json'))
print('$tag', round(j['ms_per_step'],3), [(k['kind'],k['side'],k['d'],round(k['avg_ms'],3)) for k in j['roofline_per_kernel'] if k['kind']=='adam'])"
}
NOPF="BBGR_LIB=$PWD/beyond-binary-fake-user-detection-a-credibility-aware-graph-based-recommender-system_amd/lib/ab/nopf/libbbgr.so"
run pf1 "" && run nopf1 "" $NOPF && run pf2 "" && run nopf2 "" $NOPF && \
run c3pf "--config C3 --variant cu_fair" && run c3nopf "--config C3 --variant cu_fair" $NOPF && echo ALL_OK
