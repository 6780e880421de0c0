"""Probe: run-to-run spread of bench.py's cpu_baseline leg on the GPU box's
host, with the process free to run on any CPU (the default) or pinned to the
first N CPUs of one NUMA node (--pin).

    python tools/probes/cpu_baseline_probe.py [--runs 3] [--pin 0|16]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from bbgr.synthetic import CONFIGS, CONFIG_SEED, config_edges, synthetic_credibility  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--pin", type=int, default=0)
    a = ap.parse_args()
    if a.pin:
        os.sched_setaffinity(0, set(sorted(os.sched_getaffinity(0))[:a.pin]))
    cfg = CONFIGS["C4"]
    edges = config_edges("C4")
    cred = synthetic_credibility(cfg["num_users"], CONFIG_SEED["C4"])
    for r in range(a.runs):
        t0 = time.perf_counter()
        c = bench.cpu_baseline(edges, cfg, "C4", cred, whole_steps=())
        print(json.dumps({"pin": a.pin, "run": r, "step_s": 1.0 / c["bpr_steps_per_s"],
                          "components_s": c["components_s"], "cores": c["cores"],
                          "wall_s": time.perf_counter() - t0}), flush=True)


if __name__ == "__main__":
    main()
