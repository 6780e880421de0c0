#!/bin/bash
# Round-end measurement on the GPU box: smoke, the default bench line twice
# (the CPU baseline's run-to-run spread), the C2 line, and the three
# rocprofv3 passes of the default bench command (tools/profile_box.sh).
set -o pipefail
mkdir -p gpurun_out
T=${1:-final}
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
for k in 1 2; do
  timeout -k 10 400 python bench.py > gpurun_out/${T}_bench$k.json 2> gpurun_out/${T}_bench$k.log || { echo BENCH${k}_FAILED; tail -20 gpurun_out/${T}_bench$k.log; exit 1; }
done
timeout -k 10 200 python bench.py --config C2 --steps 300 --warmup 20 > gpurun_out/${T}_c2.json 2> gpurun_out/${T}_c2.log || { echo C2_FAILED; tail -20 gpurun_out/${T}_c2.log; exit 1; }
timeout -k 10 300 python tools/dropin_probe.py --adam bbgr > gpurun_out/${T}_dropin_bbgr.json 2> gpurun_out/${T}_dropin_bbgr.log || { echo DROPIN_FAILED; tail -20 gpurun_out/${T}_dropin_bbgr.log; exit 1; }
bash tools/profile_box.sh $T || { echo PROFILE_FAILED; exit 1; }
echo ALL_OK
