"""Probe: does a degree-ordered vertex numbering speed up the C4 training step?

The synthetic graphs number items (and users) at random, as real id spaces
are. Relabelling rows by descending degree (here on the host, before the
graph is built with vertex_order="input") packs the heavily gathered rows of
each table into one address range. The step is permutation-equivariant, so
only the time changes. (The streamed-cold-row A/B of DESIGN §3 ran an earlier
form of this probe with the stream threshold set per run.)

    python tools/probes/relabel_probe.py [--steps 10] [--modes none,items,users,both]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import bbgr  # noqa: E402,F401
from bbgr import propagate as P  # noqa: E402
from bbgr.graph import BipartiteGraph  # noqa: E402
from bbgr.synthetic import CONFIGS, CONFIG_SEED, config_edges, synthetic_credibility  # noqa: E402
from bbgr.trainer import FusedTrainer  # noqa: E402


def degree_order(ids: np.ndarray, n: int) -> np.ndarray:
    """new id of each old id: rank in descending degree (stable)."""
    deg = np.bincount(ids, minlength=n)
    order = np.argsort(-deg, kind="stable")
    new = np.empty(n, np.int64)
    new[order] = np.arange(n)
    return new


def run(edges, cfg, cred, steps, warmup):
    U, I, d, K, B = (cfg[k] for k in ("num_users", "num_items", "emb_dim", "num_layers", "batch"))
    g = BipartiteGraph(edges, U, I, "cuda")
    tr = FusedTrainer(g, "v2_pop", cred=cred, emb_dim=d, num_layers=K, batch_size=B)
    for _ in range(warmup):
        tr.step()
    timer = P.SpmmTimer()
    torch.cuda.synchronize()
    P.set_spmm_timer(timer)
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    P.set_spmm_timer(None)
    seq = {k: [round(ms, 4) for _, _, ms in timer.sequence(k, steps)]
           for k in ("full", "adam", "masked")}
    del tr, g
    torch.cuda.empty_cache()
    return 1000 * el / steps, seq


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--modes", default="none,items,users,both")
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    U, I = cfg["num_users"], cfg["num_items"]
    e0 = config_edges(a.config)
    cred0 = synthetic_credibility(U, CONFIG_SEED[a.config])
    for mode in a.modes.split(","):
        e = e0.copy()
        cred = cred0
        if mode in ("items", "both"):
            e[1] = degree_order(e0[1], I)[e0[1]]
        if mode in ("users", "both"):
            nu = degree_order(e0[0], U)
            e[0] = nu[e0[0]]
            cred = np.empty_like(cred0)
            cred[nu] = cred0
        ms, seq = run(e, cfg, cred, a.steps, a.warmup)
        print(json.dumps({"mode": mode, "ms_per_step": round(ms, 3), **seq}), flush=True)


if __name__ == "__main__":
    main()
