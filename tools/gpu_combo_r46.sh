mkdir -p gpurun_out
timeout -k 10 250 python tools/dropin_probe.py --adam bbgr > gpurun_out/po_in.json 2>gpurun_out/po_in.log && timeout -k 10 250 python tools/dropin_probe.py --adam bbgr --pre-ordered > gpurun_out/po_deg.json 2> gpurun_out/po_deg.log && cat gpurun_out/po_in.json gpurun_out/po_deg.json && bash tools/gpu_round_end.sh r46
