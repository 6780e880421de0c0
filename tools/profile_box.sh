#!/bin/bash
# Runs on the GPU box from the repo root. Three rocprofv3 passes over the same
# bench command: (1) kernel trace + stats, (2) FETCH_SIZE, (3) WRITE_SIZE
# (separate PMC passes: FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2).
# Usage: tools/profile_box.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:-r01}; shift || true
ARGS=${@:---steps 5 --warmup 2 --no-cpu-baseline --no-torch-reference --dense-check 0}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export BBGR_PROFILE_MARKS=1
echo "${BBGR_COMMIT:-unknown}" > $OUT/commit.txt   # set by the caller: the box has no .git
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run \
  -- python3 bench.py $ARGS > $OUT/trace_bench.json 2> $OUT/trace_bench.log
# every kernel (no include filter): profiles/step_traffic.json sums a whole step
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/fetch -o run \
  -- python3 bench.py $ARGS > $OUT/fetch_bench.json 2> $OUT/fetch_bench.log
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/write -o run \
  -- python3 bench.py $ARGS > $OUT/write_bench.json 2> $OUT/write_bench.log
find $OUT -name "*.csv" | head -50
