#!/bin/bash
# Round 3 measurement pass on one box: the drop-in step under a kernel trace,
# the C1 (lightgcn.py symmetric path, --variant plain) and C3 (lightgcn_cu.py
# Jacobi, --variant cu_fair) bench lines with their CPU baselines.
set -o pipefail
T=${1:-r3m}
mkdir -p gpurun_out/$T
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/$T/dropin_trace -o run \
  -- python3 tools/dropin_probe.py --adam bbgr --steps 5 --warmup 2 > gpurun_out/$T/dropin_trace.json 2> gpurun_out/$T/dropin_trace.log || { echo FAIL_trace; tail -20 gpurun_out/$T/dropin_trace.log; exit 1; }
echo trace-ok
timeout -k 10 300 python -u bench.py --config C1 --variant plain > gpurun_out/$T/c1_bench.json 2> gpurun_out/$T/c1_bench.log || { echo FAIL_c1; tail -20 gpurun_out/$T/c1_bench.log; exit 1; }
echo c1-ok
timeout -k 10 600 python -u bench.py --config C3 --variant cu_fair --no-torch-reference > gpurun_out/$T/c3_bench.json 2> gpurun_out/$T/c3_bench.log || { echo FAIL_c3; tail -20 gpurun_out/$T/c3_bench.log; exit 1; }
echo OK
