"""Probe: one rank's share of the user-row-sharded step, alone on one GPU.

Rank 0 of an N-way strong split of the config's graph (edge-balanced user
range, global batch / N users per step) runs as a world-size-1 RCCL
ShardedTrainer: its collectives are local copies, so the time is the rank's
compute plus the exchange machinery's launch / range overheads without the
wire time (DESIGN §6 model: compute(N)). Swept over exchange_parts. C5 (500M
edges) is drawn per user shard (synthetic.shard_edges_strong, bench.py's N > 1
form), so rank 0's 62.5M-edge share never needs the whole graph.

    python tools/shard_probe.py [--config C4] [--parts-of 8] [--exchange-parts 1,2,4,8]
                                [--column-chains 1,2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bbgr  # noqa: E402,F401
from bbgr.distributed import ShardedTrainer, partition_users, shard_edges  # noqa: E402
from bbgr.synthetic import CONFIGS, CONFIG_SEED, config_edges, synthetic_credibility  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--parts-of", type=int, default=8)
    ap.add_argument("--exchange-parts", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--column-chains", default="1")
    ap.add_argument("--frontier-parts", default="2")
    ap.add_argument("--own-items-of", type=int, default=None,
                    help="item rows owned per rank as at world size N (default: --parts-of): "
                         "the probe's rank runs the item Adam on I/N rows, as an N-rank step "
                         "does (at world size 1 it would own every row)")
    ap.add_argument("--native-comm", default="off", choices=["off", "stream", "inline"],
                    help="the exchange through the C ABI's RCCL communicator: on a comm "
                         "stream, or every collective inline on the compute stream")
    ap.add_argument("--profile", default="",
                    help="cProfile the timed steps into <this>.c<chains>x<parts>f<fparts>")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29581")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    c = CONFIGS[a.config]
    U, I, d, K, B = (c[k] for k in ("num_users", "num_items", "emb_dim", "num_layers", "batch"))
    if c["num_edges"] > 100_000_000:
        # C5: drawn per user shard as bench.py does at N > 1 (shard_edges_strong):
        # rank 0's users and edges only, never the whole 500M-edge graph
        from bbgr.synthetic import shard_edges_strong
        local, lo, hi = shard_edges_strong(a.config, 0, a.parts_of)
        cred = synthetic_credibility(hi - lo, CONFIG_SEED[a.config])
    else:
        e = config_edges(a.config)
        deg_u = np.bincount(e[0].astype(np.int64), minlength=U)
        bounds = partition_users(deg_u, a.parts_of)
        lo, hi = int(bounds[0]), int(bounds[1])
        local = shard_edges(e, lo, hi)
        cred = synthetic_credibility(U, CONFIG_SEED[a.config])[lo:hi]
        del e
    runs = [(int(x), int(ch), int(fp)) for ch in a.column_chains.split(",")
            for x in a.exchange_parts.split(",") for fp in a.frontier_parts.split(",")]
    for xp, chains, fparts in runs:
        torch.cuda.reset_peak_memory_stats()
        tr = ShardedTrainer(local, hi - lo, I, "v2_pop", cred=cred, emb_dim=d, num_layers=K,
                            batch_size=max(1, B // a.parts_of), device="cuda",
                            vertex_order="degree", exchange_parts=xp,
                            overlap_item_adam=True, column_chains=chains,
                            frontier_parts=fparts,
                            native_comm={"off": False, "stream": True,
                                         "inline": "inline"}[a.native_comm])
        own = a.parts_of if a.own_items_of is None else a.own_items_of
        if own > 1 and tr.own_items:   # an N-rank step's item Adam share (rows [0, I/N))
            n = I // own
            tr.ia, tr.ib = 0, n
            tr.m_i, tr.v_i = tr.m_i[:n].clone(), tr.v_i[:n].clone()
        for _ in range(3):
            tr.step()
        torch.cuda.synchronize()
        prof = None
        if a.profile:   # host profile of the timed steps only
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        t0 = time.perf_counter()
        issue = 0.0
        for _ in range(a.steps):
            t1 = time.perf_counter()
            tr.step()
            issue += time.perf_counter() - t1   # host time to enqueue one step
        torch.cuda.synchronize()
        ms = 1000.0 * (time.perf_counter() - t0) / a.steps
        if prof is not None:
            prof.disable()
            prof.dump_stats(f"{a.profile}.c{chains}x{xp}f{fparts}")
        print(json.dumps({"config": a.config, "rank_of": a.parts_of, "users": hi - lo,
                          "edges": int(local.shape[1]), "exchange_parts": xp,
                          "column_chains": chains, "frontier_parts": fparts,
                          "native_comm": a.native_comm,
                          "item_rows_owned": tr.ib - tr.ia,
                          "ms_per_step": ms, "host_issue_ms": 1000.0 * issue / a.steps,
                          # device memory one such rank holds at its peak (whether
                          # N ranks of it fit one GPU for a gloo rehearsal)
                          "peak_allocated_gib": torch.cuda.max_memory_allocated() / 2**30}),
              flush=True)
        tr.close()
        del tr
        torch.cuda.empty_cache()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
