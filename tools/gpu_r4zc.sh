#!/bin/bash
# The other configs' bench lines at the final round-4 commit (tools/gpu_r4_measure.sh
# "configs", split so each call stays short): $1 = small (C1, C2, C3) | big (C5).
set -o pipefail
O=gpurun_out/r4zc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "FAIL $1"; tail -30 "$2"; exit 1; }
if [ "$1" = small ]; then
  timeout -k 10 300 python -u bench.py --config C1 --variant plain > $O/c1_bench.json 2> $O/c1_bench.log || fail c1 $O/c1_bench.log
  timeout -k 10 300 python -u bench.py --config C2 > $O/c2_bench.json 2> $O/c2_bench.log || fail c2 $O/c2_bench.log
  timeout -k 10 600 python -u bench.py --config C3 --variant cu_fair --no-torch-reference > $O/c3_bench.json 2> $O/c3_bench.log || fail c3 $O/c3_bench.log
else
  timeout -k 10 900 python -u bench.py --config C5 --steps 5 --warmup 2 --no-torch-reference --dense-check 0 > $O/c5_bench.json 2> $O/c5_bench.log || fail c5 $O/c5_bench.log
fi
for f in $O/c*_bench.json; do python3 -c "
import json; j=json.load(open('$f')); r=j['roofline']; c=j.get('cpu_baseline') or {}
print('$f', round(j['ms_per_step'],4), round(r['frac'],3), c.get('value'), c.get('unit'))"; done
echo ALL_DONE
