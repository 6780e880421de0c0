"""Probe: SpMM load-balance chunk size vs graph size (C2 / C4 training step).

Rows longer than long_threshold are cut into chunks of <= chunk_edges edges,
one workgroup each; a chunk's 16 lane groups walk its edges in 16-edge
batches, so a big chunk is a long dependent chain. On a small graph the few
hot rows' chunks are the kernel's critical path.

    python tools/probes/chunk_probe.py [--config C2] [--chunks 2048,1024,512,256]
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
from bbgr.graph import BipartiteGraph  # noqa: E402
from bbgr.synthetic import CONFIGS, CONFIG_SEED, config_edges, synthetic_credibility  # noqa: E402
from bbgr.trainer import FusedTrainer, GraphedStep  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--chunks", default="2048,1024,512,256")
    ap.add_argument("--thresholds", default="256",
                    help="long-row thresholds (rows above are cut into chunk workgroups)")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--variant", default="v2_pop")
    ap.add_argument("--graph", action="store_true", help="replay the step as a HIP graph")
    a = ap.parse_args()
    c = CONFIGS[a.config]
    U, I, d, K, B = (c[k] for k in ("num_users", "num_items", "emb_dim", "num_layers", "batch"))
    e = config_edges(a.config)
    cred = synthetic_credibility(U, CONFIG_SEED[a.config])
    for ch, thr in ((int(x), int(t)) for x in a.chunks.split(",")
                    for t in a.thresholds.split(",")):
        g = BipartiteGraph(e, U, I, "cuda", vertex_order="degree", chunk_edges=ch,
                           long_threshold=thr)
        tr = FusedTrainer(g, a.variant, cred=cred, emb_dim=d, num_layers=K, batch_size=B)
        step = GraphedStep(tr).step if a.graph else tr.step
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        print(json.dumps({"config": a.config, "variant": a.variant, "graph": a.graph,
                          "chunk_edges": ch, "long_threshold": thr,
                          "item_chunks": g.item_csr.n_chunks, "user_chunks": g.user_csr.n_chunks,
                          "ms_per_step": round(1000 * (time.perf_counter() - t0) / a.steps, 4)}),
              flush=True)
        del tr, g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
