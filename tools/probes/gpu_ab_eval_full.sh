#!/bin/bash
# A/B of evaluation builds (tools/probes/build_variant.sh with SRC=eval):
# tools/bench_eval.py through BBGR_LIB — full ranking at 262k users, or the
# sampled protocol over every test user with MODE=sampled — after the eval
# parity tests against the first variant.
# Usage: [MODE=sampled] [EVAL_ARGS="--ks 32"] tools/probes/gpu_ab_eval_full.sh <out dir> <variant> [variant ...]
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
if [ "${MODE:-full}" = sampled ]; then PROTO=""; else PROTO="--full --max-users 262144"; fi
P=beyond-binary-fake-user-detection-a-credibility-aware-graph-based-recommender-system_amd/lib/ab
BBGR_LIB=$PWD/$P/$1/libbbgr.so timeout -k 10 300 python -u -m pytest tests/test_gpu_eval.py -x -q --timeout 120 --timeout-method thread > $O/$1_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/$1_tests.log; exit 1; }
for rep in 1 2; do
  for v in "$@"; do
    BBGR_LIB=$PWD/$P/$v/libbbgr.so timeout -k 10 300 python -u tools/bench_eval.py $PROTO --reps 3 --warmup 1 --no-cpu-baseline $EVAL_ARGS >> $O/$v.jsonl 2>> $O/$v.log || { echo "BENCH $v FAILED"; exit 1; }
    echo "$v done"
  done
done
