mkdir -p gpurun_out/shvar
A="--sharded --steps 15 --no-cpu-baseline --dense-check 0"
for r in 1 2 3; do
timeout -k 10 200 python bench.py $A > gpurun_out/shvar/def_$r.json 2>/dev/null || exit 1
BBGR_EXP_NOTIMER=1 timeout -k 10 200 python bench.py $A > gpurun_out/shvar/notimer_$r.json 2>/dev/null || exit 1
BBGR_EXP_SYNC=1 timeout -k 10 200 python bench.py $A > gpurun_out/shvar/sync_$r.json 2>/dev/null || exit 1
done
for f in gpurun_out/shvar/*.json; do python -c "import json,sys;j=json.load(open('$f'));print('$f', round(j['ms_per_step'],2))"; done
