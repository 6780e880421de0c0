"""Worker for tests/test_gpu_distributed.py (launched by torch.distributed.run):
two gloo ranks share cuda:0 and run ShardedTrainer steps; each rank dumps its
state for the parent test to check against the oracle."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bbgr  # noqa: E402,F401
from bbgr.distributed import ShardedTrainer  # noqa: E402


def main():
    out_dir, variant = sys.argv[1], sys.argv[2]
    g = np.load(os.path.join(ROOT, "tests", "golden", "golden_small.npz"))
    U, I, E, DUP, D, K, B = (int(x) for x in g["meta"])
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    torch.cuda.set_device(0)
    tr = ShardedTrainer(g["edges"], U, I, variant, cred=g["cred"], emb_dim=D, num_layers=K,
                        batch_size=64, device="cuda:0", u0=g["u0"], i0=g["i0"],
                        lambda_fair=0.05 if variant == "cu_fair" else 0.0)
    loss = float(tr.step())
    users = tr.perm[: tr.B_local]          # the first step takes the head of epoch 1
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), lo=tr.lo, hi=tr.hi,
             users=users.cpu().numpy() + tr.lo, pos=tr.pos.cpu().numpy(),
             neg=tr.neg.cpu().numpy(), g_u0=tr.g_u0.cpu().numpy(), g_i0=tr.g_i0.cpu().numpy(),
             user_w=tr.user_w.cpu().numpy(), item_w=tr.item_w.cpu().numpy(), loss=loss,
             uf=tr.uf.cpu().numpy(), itf=tr.itf.cpu().numpy())
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
