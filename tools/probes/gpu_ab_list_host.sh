#!/bin/bash
# The list tests on the GPU, then A/B of host-length frontier lists
# (BBGR_LIST_HOST=1, the default) vs the device count (0) on the C4 bench.
set -o pipefail
O=gpurun_out/${1:-ablisthost}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "host_length or frontier_step or fused_adam_step" tests/test_gpu_graph.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for rep in 1 2; do
for lh in 0 1; do
  BBGR_LIST_HOST=$lh timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-torch-reference --dense-check 0 > $O/lh${lh}_$rep.json 2> $O/lh${lh}_$rep.log || { tail -20 $O/lh${lh}_$rep.log; exit 1; }
  python3 -c "
import json; j=json.load(open('$O/lh${lh}_$rep.json')); m=j['frontier']['masked_sequence_ms']
print('$lh', round(j['ms_per_step'],3), [round(x['avg_ms'],4) for x in m])"
done; done
echo ALL_DONE
