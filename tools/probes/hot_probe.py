"""Probe: size of the hot (cached) prefix of each gathered / written table in
degree order (graph.HOT_BYTES and the rows/8 cap), on one C4 trainer. The
rule is swapped between runs on the same trainer (it is evaluated per launch).

    python tools/probes/hot_probe.py [--steps 15] [--cases 8:8:192,8:64:192]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bbgr  # noqa: E402,F401
from bbgr import graph as G  # noqa: E402
from bbgr.graph import BipartiteGraph  # noqa: E402
from bbgr.synthetic import CONFIGS, CONFIG_SEED, config_edges, synthetic_credibility  # noqa: E402
from bbgr.trainer import FusedTrainer  # noqa: E402


def rule(user_div, item_div, budget_mb, U):
    def hot(n, d):
        div = user_div if n == U else item_div
        if div <= 0:
            return 0
        return max(1, min(n // div, (budget_mb << 20) // (4 * d)))

    def stream_from(self, d):
        return hot(self.n_cols, d) if self.__dict__.get("cols_by_degree") else 0

    def stream_out_from(self, d):
        return hot(self.n_rows, d) if self.__dict__.get("rows_by_degree") else 0
    return stream_from, stream_out_from


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=15)
    ap.add_argument("--cases", default="",
                    help="user_div:item_div:budget_mb,... (default: the round-2 sweep)")
    a = ap.parse_args()
    c = CONFIGS["C4"]
    U, I, d, K, B = (c[k] for k in ("num_users", "num_items", "emb_dim", "num_layers", "batch"))
    g = BipartiteGraph(config_edges("C4"), U, I, "cuda", vertex_order="degree")
    tr = FusedTrainer(g, "v2_pop", cred=synthetic_credibility(U, CONFIG_SEED["C4"]), emb_dim=d,
                      num_layers=K, batch_size=B)
    cases = [(8, 8, 192), (8, 4, 192), (8, 2, 192), (16, 8, 192), (4, 8, 256), (8, 1, 256),
             (0, 0, 0), (8, 8, 192)]
    if a.cases:
        cases = [tuple(int(v) for v in c.split(":")) for c in a.cases.split(",")]
    for ud, idv, mb in cases:
        G.Csr.stream_from, G.Csr.stream_out_from = rule(ud, idv, mb, U)
        for _ in range(3):
            tr.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            tr.step()
        torch.cuda.synchronize()
        ms = 1000 * (time.perf_counter() - t0) / a.steps
        print(json.dumps({"user_div": ud, "item_div": idv, "budget_mb": mb,
                          "ms_per_step": round(ms, 3)}), flush=True)


if __name__ == "__main__":
    main()
