mkdir -p gpurun_out/shvar2
A="--sharded --steps 15 --no-cpu-baseline"
for r in 1 2; do
timeout -k 10 200 python bench.py $A > gpurun_out/shvar2/sh_$r.json 2>/dev/null || exit 1
done
timeout -k 10 200 python bench.py --steps 15 --no-cpu-baseline > gpurun_out/shvar2/fused.json 2>/dev/null || exit 1
BBGR_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/shvar2/gloo2.json 2> gpurun_out/shvar2/gloo2.log || { echo GLOO2_FAILED; tail -20 gpurun_out/shvar2/gloo2.log; exit 1; }
for f in gpurun_out/shvar2/*.json; do python -c "import json;j=json.load(open('$f'));print('$f', round(j['ms_per_step'],2), j['dense_ms_per_step'], round(j['roofline']['frac'],3), j['roofline']['events'], j['scaling'], j['n_gpus'])"; done
