#!/bin/bash
# Round-4 measurement pass on one GPU box (from the repo root):
#   configs  C1 / C2 / C3 / C5 bench lines at HEAD (C5: no CPU baseline)
#   profile  rocprofv3 kernel trace + FETCH_SIZE + WRITE_SIZE passes of the C4 bench
#   shard    the N=8 user-row rank probe (1 and 2 column chains)
#   dropin   the drop-in module step (FusedAdam / foreach Adam)
#   rehearsal the driver's N=4 / N=8 bench commands over gloo on one GPU
# Usage: tools/gpu_r4_measure.sh <tag> <pass>...   outputs under gpurun_out/<tag>/
set -o pipefail
T=${1:-r4m}; shift
O=gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "FAIL $1"; tail -30 "$2"; exit 1; }
for WHAT in "$@"; do
case $WHAT in
configs)
  timeout -k 10 300 python -u bench.py --config C1 --variant plain > $O/c1_bench.json 2> $O/c1_bench.log || fail c1 $O/c1_bench.log
  timeout -k 10 300 python -u bench.py --config C2 > $O/c2_bench.json 2> $O/c2_bench.log || fail c2 $O/c2_bench.log
  timeout -k 10 600 python -u bench.py --config C3 --variant cu_fair --no-torch-reference > $O/c3_bench.json 2> $O/c3_bench.log || fail c3 $O/c3_bench.log
  timeout -k 10 600 python -u bench.py --config C5 --steps 5 --warmup 2 --no-torch-reference --dense-check 0 > $O/c5_bench.json 2> $O/c5_bench.log || fail c5 $O/c5_bench.log
  ;;
profile)
  timeout -k 10 1000 bash tools/profile_box.sh $T > $O/profile.log 2>&1 || fail profile $O/profile.log
  ;;
shard)
  timeout -k 10 300 python -u tools/shard_probe.py --exchange-parts 1 --column-chains 1,2 --frontier-parts 1 > $O/shard8.jsonl 2> $O/shard8.log || fail shard $O/shard8.log
  cat $O/shard8.jsonl
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/shard8_trace -o run -- python3 tools/shard_probe.py --exchange-parts 1 --column-chains 1 --frontier-parts 1 --steps 10 > $O/shard8_trace.jsonl 2> $O/shard8_trace.log || fail shardtrace $O/shard8_trace.log
  ;;
dropin)
  timeout -k 10 300 python tools/dropin_probe.py --adam bbgr > $O/dropin_bbgr.json 2> $O/dropin_bbgr.log || fail dropin $O/dropin_bbgr.log
  timeout -k 10 300 python tools/dropin_probe.py --adam foreach > $O/dropin_foreach.json 2> $O/dropin_foreach.log || fail dropin_foreach $O/dropin_foreach.log
  ;;
rehearsal)   # the driver's N=4 / N=8 bench commands over gloo on this one GPU
  timeout -k 10 1000 bash tools/probes/gpu_rehearsal_n48.sh ${T}/rehearsal > $O/rehearsal.log 2>&1 || fail rehearsal $O/rehearsal.log
  cat $O/rehearsal.log
  ;;
*) echo "unknown pass $WHAT"; exit 2 ;;
esac
echo "PASS $WHAT ok"
done
echo ALL_OK
