set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4s
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ops.py tests/test_gpu_lazy.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4s/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4s/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r4s/tests.log | head; exit 1; }
timeout -k 10 300 python tools/dropin_probe.py --adam bbgr > gpurun_out/r4s/dropin_bbgr.json 2> gpurun_out/r4s/dropin_bbgr.log || { tail -20 gpurun_out/r4s/dropin_bbgr.log; exit 1; }
timeout -k 10 300 python tools/dropin_probe.py --adam foreach > gpurun_out/r4s/dropin_foreach.json 2> gpurun_out/r4s/dropin_foreach.log || { tail -20 gpurun_out/r4s/dropin_foreach.log; exit 1; }
for t in bbgr foreach; do python -c "import json; j=json.load(open('gpurun_out/r4s/dropin_$t.json')); print('$t', {k: round(j[k],3) for k in ('step_ms','forward_ms','forward_backward_ms','adam_ms')})"; done
echo ALL_OK
