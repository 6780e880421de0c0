"""Probe: the reference's training step in STOCK PyTorch-ROCm on the same
MI355X (measurement tool, not product, not the oracle): the V2 step written
with the torch calls the reference makes — COO operators built with
sparse_coo_tensor(...).coalesce() (Version-2/lighgcn_cu_pop.py:441-450),
torch.sparse.mm per layer in Gauss-Seidel order and stack().mean(0)
(:482-489), the BPR + ego-L2 loss (:496-507), loss.backward() and
torch.optim.Adam(lr=1e-3) (:793, :858-863) — all on cuda. This is what the
reference's own code does on this GPU, the like-for-like GPU baseline for
the HIP path (bench.py / tools/dropin_probe.py). Batches are uniform draws
made up front (the sampler is not what this times). variant="cu_fair" runs
lightgcn_cu.py's step instead: its operators (`lightgcn_cu.py:383-397`,
credibility on the item<-user side, 1/sqrt(deg_u*deg_i)), Jacobi layers
(:429-447) and the fairness term (:583-584, 637-648).

    python tools/torch_sparse_step.py [--config C4] [--steps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bbgr  # noqa: E402,F401
from bbgr.synthetic import CONFIGS, CONFIG_SEED, config_edges, synthetic_credibility  # noqa: E402


def operators_cu(e: np.ndarray, U: int, I: int, cred: torch.Tensor, dev):
    """(item<-user [I,U], user<-item [U,I], deg_i) of lightgcn_cu.py."""
    u = torch.as_tensor(e[0], dtype=torch.int64, device=dev)
    i = torch.as_tensor(e[1], dtype=torch.int64, device=dev)
    du = torch.bincount(u, minlength=U).float()
    di = torch.bincount(i, minlength=I).float()
    w = 1.0 / torch.sqrt(torch.clamp(du[u] * di[i], min=1e-12))
    M_item = torch.sparse_coo_tensor(torch.stack([i, u]), cred[u] * w, (I, U)).coalesce()
    M_user = torch.sparse_coo_tensor(torch.stack([u, i]), w, (U, I)).coalesce()
    return M_item, M_user, di


def operators(e: np.ndarray, U: int, I: int, cred: torch.Tensor, dev):
    u = torch.as_tensor(e[0], dtype=torch.int64, device=dev)
    i = torch.as_tensor(e[1], dtype=torch.int64, device=dev)
    du = torch.bincount(u, minlength=U).clamp(min=1).float()
    di = torch.bincount(i, minlength=I).clamp(min=1).float()
    w = du[u].rsqrt() * di[i].rsqrt()
    M_ui = torch.sparse_coo_tensor(torch.stack([u, i]), w, (U, I)).coalesce()
    M_iu = torch.sparse_coo_tensor(torch.stack([i, u]), cred[u] * w, (I, U)).coalesce()
    return M_ui, M_iu


class Model(torch.nn.Module):
    def __init__(self, U, I, d, K, M_ui, M_iu, jacobi: bool = False, pop=None,
                 lambda_fair: float = 0.0):
        super().__init__()
        self.K, self.M_ui, self.M_iu = K, M_ui, M_iu
        self.jacobi, self.pop, self.lambda_fair = jacobi, pop, lambda_fair
        self.user_emb = torch.nn.Embedding(U, d)
        self.item_emb = torch.nn.Embedding(I, d)
        torch.nn.init.xavier_uniform_(self.user_emb.weight)
        torch.nn.init.xavier_uniform_(self.item_emb.weight)

    def propagate(self):
        u = self.user_emb.weight
        i = self.item_emb.weight
        us, is_ = [u], [i]
        for _ in range(self.K):
            if self.jacobi:   # both from the previous layer (M_iu: item<-user here)
                i, u = torch.sparse.mm(self.M_iu, us[-1]), torch.sparse.mm(self.M_ui, is_[-1])
            else:
                i = torch.sparse.mm(self.M_iu, u)
                u = torch.sparse.mm(self.M_ui, i)
            us.append(u)
            is_.append(i)
        return torch.stack(us, 0).mean(0), torch.stack(is_, 0).mean(0)

    def bpr_loss(self, users, pos, neg, uf, itf, reg):
        u, p, n = uf[users], itf[pos], itf[neg]
        x = (u * p).sum(1) - (u * n).sum(1)
        loss = -torch.log(torch.sigmoid(x) + 1e-12).mean()
        ue, ie = self.user_emb.weight, self.item_emb.weight
        r = (ue[users].norm(2, dim=1).pow(2) + ie[pos].norm(2, dim=1).pow(2)
             + ie[neg].norm(2, dim=1).pow(2)).mean()
        loss = loss + reg * r
        if self.pop is not None:
            loss = loss + self.lambda_fair * (self.pop[pos] * (u * p).sum(1)).mean()
        return loss


def timed(fn, steps: int) -> float:
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return 1000.0 * (time.perf_counter() - t0) / steps


def run(cfg_name: str, edges: np.ndarray | None = None, cred_np=None, steps: int = 5,
        warmup: int = 2, device=None, variant: str = "v2_pop") -> dict:
    """Times of the stock-torch reference step at `cfg_name` (edges / cred
    drawn if not given). Frees its tensors before returning."""
    c = CONFIGS[cfg_name]
    U, I, d, K, B = (c[k] for k in ("num_users", "num_items", "emb_dim", "num_layers", "batch"))
    dev = torch.device(device) if device is not None else torch.device("cuda")
    e = config_edges(cfg_name) if edges is None else edges
    if cred_np is None:
        cred_np = synthetic_credibility(U, CONFIG_SEED[cfg_name])
    cred = torch.as_tensor(np.asarray(cred_np, np.float32), device=dev)
    t0 = time.perf_counter()
    torch.manual_seed(42)
    if variant == "cu_fair":
        M_item, M_user, di = operators_cu(e, U, I, cred, dev)
        model = Model(U, I, d, K, M_user, M_item, jacobi=True,
                      pop=di / di.max().clamp(min=1.0), lambda_fair=0.05).to(dev)
    else:
        M_ui, M_iu = operators(e, U, I, cred, dev)
        model = Model(U, I, d, K, M_ui, M_iu).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0
    g = torch.Generator(device=dev).manual_seed(1)
    n_b = warmup + steps
    users = torch.randint(0, U, (n_b, B), device=dev, generator=g)
    pos = torch.randint(0, I, (n_b, B), device=dev, generator=g)
    neg = torch.randint(0, I, (n_b, B), device=dev, generator=g)
    it = iter(range(10**9))

    def fwd_bwd():
        k = next(it) % n_b
        uf, itf = model.propagate()
        loss = model.bpr_loss(users[k], pos[k], neg[k], uf, itf, 1e-4)
        opt.zero_grad()
        loss.backward()

    def step():
        fwd_bwd()
        opt.step()

    def fwd():
        with torch.no_grad():
            model.propagate()

    for _ in range(warmup):
        step()
    out = {"config": cfg_name, "variant": "cu_fair" if variant == "cu_fair" else "v2_pop",
           "torch": torch.__version__, "setup_s": setup_s,
           "num_edges": int(e.shape[1]), "steps": steps,
           "step_ms": timed(step, steps), "forward_ms": timed(fwd, steps),
           "forward_backward_ms": timed(fwd_bwd, steps),
           "adam_ms": timed(opt.step, steps)}
    out["edges_per_s_4KE"] = 4 * K * int(e.shape[1]) / (out["step_ms"] / 1e3)
    del model, opt, users, pos, neg
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--variant", default="v2_pop", choices=["v2_pop", "cu_fair"])
    a = ap.parse_args()
    print(json.dumps(run(a.config, steps=a.steps, warmup=a.warmup, variant=a.variant)),
          flush=True)


if __name__ == "__main__":
    main()
