"""Print the per-launch SpMM sequence of bench.py JSON lines (A/B runs)."""
import json
import sys

for f in sys.argv[1:]:
    j = json.load(open(f))
    fr = j["frontier"]

    def seq(k):
        return " ".join(f"{x['rows'] // 1000}k:{x['avg_ms']:.3f}" for x in fr.get(k, []))
    print(f"{f}: {j['ms_per_step']:.2f} ms/step frac={j['roofline']['frac']:.3f}\n"
          f"  full {seq('full_sequence_ms')}\n  adam {seq('adam_sequence_ms')}\n"
          f"  masked {seq('masked_sequence_ms')}")
