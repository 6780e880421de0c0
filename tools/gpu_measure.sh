#!/bin/bash
# Measurement passes on one GPU box (run through gpurun from the repo root):
#   tools/gpu_measure.sh <tag> dropin    drop-in module step: degree-ordered vs
#                                        input-order drop-in graph (FusedAdam),
#                                        foreach torch Adam, then a kernel trace
#   tools/gpu_measure.sh <tag> configs   C1 (--variant plain) and C3 (--variant
#                                        cu_fair) bench lines with CPU baselines
#   tools/gpu_measure.sh <tag> bench     the default bench line (C4)
# Outputs under gpurun_out/<tag>/. Every GPU step has its own time limit and
# the script stops at the first failure.
set -o pipefail
T=${1:-measure}; WHAT=${2:-bench}
O=gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "FAIL $1"; tail -20 "$2"; exit 1; }
case $WHAT in
dropin)
  for o in degree input; do
    BBGR_DROPIN_ORDER=$o timeout -k 10 300 python tools/dropin_probe.py --adam bbgr \
      > $O/dropin_bbgr_$o.json 2> $O/dropin_bbgr_$o.log || fail dropin_$o $O/dropin_bbgr_$o.log
    cat $O/dropin_bbgr_$o.json
  done
  timeout -k 10 300 python tools/dropin_probe.py --adam foreach > $O/dropin_foreach.json \
    2> $O/dropin_foreach.log || fail dropin_foreach $O/dropin_foreach.log
  cat $O/dropin_foreach.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/dropin_trace -o run \
    -- python3 tools/dropin_probe.py --adam bbgr --steps 5 --warmup 2 > $O/dropin_trace.json \
    2> $O/dropin_trace.log || fail dropin_trace $O/dropin_trace.log
  ;;
configs)
  timeout -k 10 300 python -u bench.py --config C1 --variant plain > $O/c1_bench.json \
    2> $O/c1_bench.log || fail c1 $O/c1_bench.log
  timeout -k 10 600 python -u bench.py --config C3 --variant cu_fair --no-torch-reference \
    > $O/c3_bench.json 2> $O/c3_bench.log || fail c3 $O/c3_bench.log
  ;;
bench)
  timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.log || fail bench $O/bench.log
  ;;
*) echo "unknown pass $WHAT"; exit 2 ;;
esac
echo OK
