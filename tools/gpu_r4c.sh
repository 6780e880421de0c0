#!/bin/bash
# Round-4 full check at HEAD: the whole GPU suite (no -x: every failure is
# listed), then smoke(). A fault, abort, segfault or time limit (exit 124 /
# 134 / 137 / 139) ends the script there.
set -o pipefail
O=gpurun_out/${1:-r4c}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
hard() { case $1 in 124|134|137|139) echo "HARD FAIL ($1) in $2"; tail -30 "$3"; exit 1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --durations=15 --timeout 500 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; hard $rc tests $O/gpu_tests.log
echo "TESTS rc=$rc"; grep -E "passed|failed" $O/gpu_tests.log | tail -2; grep FAILED $O/gpu_tests.log | head -20
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; hard $rc smoke $O/smoke.log; echo "SMOKE rc=$rc"; tail -1 $O/smoke.log
echo ALL_DONE
