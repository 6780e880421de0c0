"""Probe: host issue time vs device time of one training step (C4).

Measures, per trainer (single-GPU FusedTrainer, sharded trainer at world 1
over RCCL with a few exchange_parts values):
  issue_ms  CPU time of trainer.step() with the GPU still busy (no sync), i.e.
            how fast the host can enqueue a step;
  step_ms   wall time per step over a synced loop.
If issue_ms approaches step_ms the GPU starves between launches.

    python tools/probes/host_probe.py [--parts 8,2]
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
from bbgr import propagate as P  # noqa: E402
from bbgr.graph import BipartiteGraph  # noqa: E402
from bbgr.synthetic import CONFIGS, CONFIG_SEED, config_edges, synthetic_credibility  # noqa: E402


def measure(tr, steps: int, timer: bool):
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    if timer:
        P.set_spmm_timer(P.SpmmTimer())
    issue = []
    for _ in range(3):   # issue one step while the GPU is idle -> pure host time
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.step()
        issue.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    P.set_spmm_timer(None)
    return {"issue_ms": round(1000 * min(issue), 3), "step_ms": round(1000 * el / steps, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", default="8,2")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    cfg = CONFIGS["C4"]
    U, I, d, K, B = (cfg[k] for k in ("num_users", "num_items", "emb_dim", "num_layers", "batch"))
    e = config_edges("C4")
    cred = synthetic_credibility(U, CONFIG_SEED["C4"])
    from bbgr.trainer import FusedTrainer
    g = BipartiteGraph(e, U, I, "cuda")
    tr = FusedTrainer(g, "v2_pop", cred=cred, emb_dim=d, num_layers=K, batch_size=B)
    for timer in (False, True):
        print(json.dumps({"trainer": "fused", "timer": timer, **measure(tr, a.steps, timer)}),
              flush=True)
    del tr, g
    torch.cuda.empty_cache()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29581")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", 0))
    from bbgr.distributed import ShardedTrainer
    for p in (int(x) for x in a.parts.split(",")):
        tr = ShardedTrainer(e, U, I, "v2_pop", cred=cred, emb_dim=d, num_layers=K,
                            batch_size=B, device="cuda:0", exchange_parts=p)
        for timer in (False, True):
            print(json.dumps({"trainer": f"sharded p{p}", "timer": timer,
                              **measure(tr, a.steps, timer)}), flush=True)
        del tr
        torch.cuda.empty_cache()
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
