#!/bin/bash
# Round 4: where the N=8 user-row rank's step goes — host profile (cProfile of
# the timed steps) and a kernel trace cut into steps (tools/step_timeline.py).
set -o pipefail
O=gpurun_out/${1:-r4e}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/shard_probe.py --exchange-parts 1 --column-chains 1 --frontier-parts 1 --profile $O/shard8.prof > $O/shard8.jsonl 2> $O/shard8.log || { tail -20 $O/shard8.log; exit 1; }
cat $O/shard8.jsonl
python - <<PY
import pstats, glob
for f in sorted(glob.glob("$O/shard8.prof.*")):
    print("==", f)
    pstats.Stats(f).sort_stats("tottime").print_stats(30)
    pstats.Stats(f).sort_stats("cumulative").print_stats(40)
PY
timeout -k 10 300 rocprofv3 --kernel-trace -T --output-format csv -d $O/trace -o run -- python3 tools/shard_probe.py --exchange-parts 1 --column-chains 1 --frontier-parts 1 --steps 10 > $O/trace.jsonl 2> $O/trace.log || { tail -20 $O/trace.log; exit 1; }
python tools/step_timeline.py $(find $O/trace -name "*kernel_trace.csv" | head -1) --steps 6 > $O/timeline.txt && head -150 $O/timeline.txt
echo ALL_OK
