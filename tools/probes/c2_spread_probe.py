"""Probe: run-to-run spread of the whole C2 reference step (bench.py
cpu_baseline) under different host-thread settings, pinned to one NUMA node.

    python tools/probes/c2_spread_probe.py [--reps 11]

One JSON line per setting: median, IQR / median, (max - min) / median."""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
argv, sys.argv = sys.argv, ["bench.py"]
import bench  # noqa: E402
sys.argv = argv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=11)
    ap.add_argument("--threads", default="16,15,12,8")
    ap.add_argument("--config", default="C2")
    a = ap.parse_args()
    cpus = sorted(os.sched_getaffinity(0))[:16]
    os.sched_setaffinity(0, cpus)
    for n in (int(x) for x in a.threads.split(",")):
        torch.set_num_threads(n)
        med, ts, work = bench._reference_step_s(a.config, "v2_pop", a.reps)
        print(json.dumps({"threads": n, "cpus": bench._cpu_list_text(cpus), "median_s": med,
                          "runs": [round(t, 4) for t in ts], **bench._spread(ts)}), flush=True)


if __name__ == "__main__":
    main()
