"""Probe: per-step wall times of the C4 training step, each step synced
(single-GPU trainer, and the sharded trainer at world 1 over RCCL), to tell
steady per-step cost from occasional stalls.

    python tools/probes/step_times.py [--steps 30]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bbgr  # noqa: E402,F401
from bbgr.graph import BipartiteGraph  # noqa: E402
from bbgr.synthetic import CONFIGS, CONFIG_SEED, config_edges, synthetic_credibility  # noqa: E402


def times(tr, n):
    for _ in range(3):
        tr.step()
    out = []
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.step()
        torch.cuda.synchronize()
        out.append(round(1000 * (time.perf_counter() - t0), 2))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    c = CONFIGS["C4"]
    U, I, d, K, B = (c[k] for k in ("num_users", "num_items", "emb_dim", "num_layers", "batch"))
    e = config_edges("C4")
    cred = synthetic_credibility(U, CONFIG_SEED["C4"])
    from bbgr.trainer import FusedTrainer
    tr = FusedTrainer(BipartiteGraph(e, U, I, "cuda", vertex_order="degree"), "v2_pop",
                      cred=cred, emb_dim=d, num_layers=K, batch_size=B)
    print(json.dumps({"trainer": "fused", "ms": times(tr, a.steps)}), flush=True)
    del tr
    torch.cuda.empty_cache()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29587")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    opts = torch.distributed.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", 0),
                                         pg_options=opts)
    from bbgr.distributed import ShardedTrainer
    tr = ShardedTrainer(e, U, I, "v2_pop", cred=cred, emb_dim=d, num_layers=K, batch_size=B,
                        device="cuda:0", exchange_parts=8, vertex_order="degree")
    print(json.dumps({"trainer": "sharded", "ms": times(tr, a.steps)}), flush=True)
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
