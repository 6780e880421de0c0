"""Probe: bbgr_adam (optim.adam_step) over the C4 item table (1M x 64) and
user table (5M x 64), HIP-event timed, with the HBM rate of its 28 B/param
(param, grad, exp_avg, exp_avg_sq in; param, exp_avg, exp_avg_sq out).

    python tools/probes/adam_probe.py [--reps 50]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bbgr  # noqa: E402,F401
from bbgr.optim import adam_step  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    out = {}
    for rows in (1_000_000, 5_000_000):
        p, g, m, v = (torch.rand(rows, 64, device="cuda") for _ in range(4))
        for _ in range(3):
            adam_step(p, g, m, v, 1, 1e-3)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for t in range(a.reps):
            adam_step(p, g, m, v, t + 2, 1e-3)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        out[f"rows_{rows}"] = {"ms": ms, "TBps": 28 * rows * 64 / (ms * 1e-3) / 1e12}
        del p, g, m, v
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
