"""Print the headline numbers of a bench.py JSON line (used by tools/gpu_run.sh).

    python tools/bench_brief.py gpurun_out/<tag>/bench.json
"""
import json
import sys


def main(path: str):
    j = json.loads(open(path).read().strip().splitlines()[-1])
    r = j["roofline"]
    print(f"ms/step {j['ms_per_step']:.3f}  value {j['value'] / 1e9:.2f} G/s  frac {r['frac']:.3f}"
          f"  dom {r['avg_launch_ms']:.4f} ms  dense {j.get('dense_ms_per_step')}"
          f"  part {j.get('partition')}  loss {j.get('final_loss')}")
    fr = j.get("frontier") or {}
    for k in ("full_sequence_ms", "adam_sequence_ms", "masked_sequence_ms"):
        seq = fr.get(k) or []
        print(f"  {k}: {[round(x['avg_ms'], 4) for x in seq]}")
    for k in ("partition_beside", "chain_beside", "weak_beside"):
        b = j.get(k)
        if b:
            print(f"  {k}: {json.dumps({x: b.get(x) for x in ('part', 'mode', 'ms_per_step', 'value')})}")
    c = j.get("cpu_baseline")
    if c:
        print(f"  cpu {c['value'] / 1e6:.2f} M/s on {c['cores']} threads: {c['sample'][:160]}")
    for k in ("dropin_module_step", "dropin_fused_adam_step", "dropin_backward_adam_step"):
        d = j.get(k)
        if d:
            print(f"  {k}: " + json.dumps({x: d.get(x) for x in
                                           ("step_ms", "forward_ms", "forward_backward_ms",
                                            "adam_ms", "optimizer")}))


if __name__ == "__main__":
    main(sys.argv[1])
