"""Probe: one column shard (ColumnShardedTrainer with column_parts=N, run
alone on one GPU: the per-rank work of an N-GPU column-sharded step) on a
BASELINE config, across long-row thresholds of the shared graph.

    python tools/probes/column_probe.py [--config C4] [--parts 2,4,8] [--thresholds 256,64,32]
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
from bbgr.columns import ColumnShardedTrainer  # noqa: E402
from bbgr.graph import BipartiteGraph  # noqa: E402
from bbgr.synthetic import CONFIGS, CONFIG_SEED, config_edges, synthetic_credibility  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--parts", default="2,4,8")
    ap.add_argument("--thresholds", default="256,64,32")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    c = CONFIGS[a.config]
    U, I, d, K, B = (c[k] for k in ("num_users", "num_items", "emb_dim", "num_layers", "batch"))
    e = config_edges(a.config)
    cred = synthetic_credibility(U, CONFIG_SEED[a.config])
    for thr in (int(t) for t in a.thresholds.split(",")):
        g = BipartiteGraph(e, U, I, "cuda", vertex_order="degree", long_threshold=thr)
        for n in (int(x) for x in a.parts.split(",")):
            tr = ColumnShardedTrainer(g, U, I, "v2_pop", cred=cred, emb_dim=d, num_layers=K,
                                      batch_size=B, column_parts=n, column_index=0, device="cuda")
            for _ in range(3):
                tr.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                tr.step()
            torch.cuda.synchronize()
            print(json.dumps({"config": a.config, "parts": n, "columns": d // n,
                              "long_threshold": thr, "item_chunks": g.item_csr.n_chunks,
                              "ms_per_step": round(1000 * (time.perf_counter() - t0) / a.steps, 4)}),
                  flush=True)
            del tr
            torch.cuda.empty_cache()
        del g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
