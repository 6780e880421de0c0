#!/bin/bash
# A/B of SpMM builds on the GPU box: bench.py with the in-tree libbbgr.so
# (base) and with each extra library given as an argument (BBGR_LIB).
# Usage: tools/probes/ab_spmm.sh [path/to/variant/libbbgr.so ...]
set -o pipefail
mkdir -p gpurun_out/ab
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/ab/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/ab/tests.log; exit 1; }
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.log || { echo "BENCH $tag FAILED"; tail -20 gpurun_out/ab/$tag.log; exit 1; }
  echo "$tag done"
}
run base
k=0
for lib in "$@"; do k=$((k+1)); run v$k BBGR_LIB=$PWD/$lib; done
echo ALL_OK
