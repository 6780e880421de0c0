#!/bin/bash
# chunk_row_serial's single-live-edge fast path: the slot-bitmap parity tests,
# then an interleaved A/B of the C4 bench against the previous spmm.hip
# (lib/ab/head, via BBGR_LIB), then the drop-in step's kernel timeline.
set -o pipefail
O=gpurun_out/${1:-abserial}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HEADLIB=$(ls -d beyond-binary-*_amd)/lib/ab/head/libbbgr.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "bitmap or slot or bits or frontier or mask or row_list or host_length or fused_adam" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for rep in 1 2; do
for v in head new; do
  if [ $v = head ]; then export BBGR_LIB=$PWD/$HEADLIB; else unset BBGR_LIB; fi
  timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-torch-reference --dense-check 0 > $O/$v$rep.json 2> $O/$v$rep.log || { tail -20 $O/$v$rep.log; exit 1; }
  python3 -c "
import json; j=json.load(open('$O/$v$rep.json')); m=j['frontier']['masked_sequence_ms']
print('$v', round(j['ms_per_step'],3), [round(x['avg_ms'],4) for x in m])"
done; done
unset BBGR_LIB
timeout -k 10 300 rocprofv3 --kernel-trace -T --output-format csv -d $O/dtrace -o run -- python3 tools/dropin_probe.py --adam bbgr --steps 6 > $O/dropin_probe.json 2> $O/dropin_probe.log || { tail -20 $O/dropin_probe.log; exit 1; }
F=$(find $O/dtrace -name "*kernel_trace.csv" | head -1)
python tools/step_timeline.py $F --marker bpr_reduce_kernel --index 5 > $O/dropin_timeline.txt || true
head -3 $O/dropin_timeline.txt
echo ALL_DONE
