"""Probe: the reference's own training step through the drop-in module API
(Version-2/lighgcn_cu_pop.py:858-863 — propagate, bpr_loss, zero_grad,
backward, torch.optim.Adam.step) on a BASELINE config, beside the fused
trainer's step on the same graph. The batches are drawn up front, as the
reference's loop draws them (`--batches reference`, the default: the epoch
shuffle of the train users and the per-user positive / pop-mix negative
draws of Version-2:821-849, through bbgr.host_sampler with the numpy
Generator seeded 42) or uniformly on the device (`--batches uniform`, the
rounds 2-5 figures); the sampler itself is not what this times.

    python tools/dropin_probe.py [--config C4] [--steps 10] [--adam foreach|fused|bbgr]

Prints one JSON line per variant: ms per step and a breakdown
(forward, forward+backward, Adam) from separately synchronised runs.
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
from bbgr import lightgcn_cu_pop as V2  # noqa: E402
from bbgr.synthetic import CONFIGS, CONFIG_SEED, config_edges, synthetic_credibility  # noqa: E402


def timed(fn, steps: int) -> float:
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return 1000.0 * (time.perf_counter() - t0) / steps


def reference_batches(edges, U: int, I: int, B: int, n_b: int, seed: int = 42,
                      gamma: float = 0.75, mix_pop: float = 0.7):
    """n_b batches of the reference's loop (Version-2:805-849): pop_prob from
    the train degrees, the shuffled train users sliced by B, a positive from
    each user's row and a pop-mix negative (bbgr.host_sampler, bit for bit
    the reference's numpy stream); int64 [n_b, B] each (a short last slice
    wraps into the next epoch's shuffle, as later epochs would)."""
    from bbgr import host_sampler as HS
    e = np.asarray(edges)
    indptr, indices = HS.edges_to_user_csr(e, U)
    deg = np.bincount(e[1].astype(np.int64), minlength=I).astype(np.float64)
    pop = np.power(deg + 1.0, gamma)
    pop_prob = pop / (pop.sum() + 1e-12)
    rng = np.random.default_rng(seed)
    train_users = np.where(np.diff(indptr) > 0)[0]
    out_u, out_p, out_n, order, at = [], [], [], np.empty(0, np.int64), 0
    while len(out_u) < n_b:
        if at + B > order.size:   # a new epoch
            rng.shuffle(train_users)
            order, at = train_users.copy(), 0
        u, p, n = HS.sample_batch(indptr, indices, order[at:at + B], I, rng, pop_prob,
                                  mix_pop=mix_pop)
        at += B
        out_u.append(u)
        out_p.append(p)
        out_n.append(n)
    return (np.stack(out_u), np.stack(out_p), np.stack(out_n))


def run(cfg_name: str, edges=None, cred_np=None, steps: int = 10, warmup: int = 3,
        adam: str = "foreach", device=None, pre_ordered: bool = False,
        items_ordered: bool = False, dense_finals: bool = False,
        batches: str = "reference") -> dict:
    """One optimizer (module docstring)."""
    return run_many(cfg_name, edges, cred_np, steps, warmup, (adam,), device, pre_ordered,
                    items_ordered, dense_finals, batches)[adam]


def run_many(cfg_name: str, edges=None, cred_np=None, steps: int = 10, warmup: int = 3,
             adams=("foreach",), device=None, pre_ordered: bool = False,
             items_ordered: bool = False, dense_finals: bool = False,
             batches: str = "reference") -> dict:
    """{adam: result} for each optimizer in `adams`, on ONE model built once
    (each optimizer starts fresh on the weights the previous one left: the
    timings do not depend on the values)."""
    c = CONFIGS[cfg_name]
    U, I, d, K, B = (c[k] for k in ("num_users", "num_items", "emb_dim", "num_layers", "batch"))
    e = config_edges(cfg_name) if edges is None else edges
    if pre_ordered:   # ids renumbered once at ingest (the graph detects the order)
        from bbgr.ingest import degree_relabel
        e = degree_relabel(e, U, I)[0]
    elif items_ordered:   # only the item ids renumbered by degree
        from bbgr.ingest import degree_relabel
        e = np.stack([np.asarray(e[0]), degree_relabel(e, U, I)[0][1]]).astype(np.int32)
    if cred_np is None:
        cred_np = synthetic_credibility(U, CONFIG_SEED[cfg_name])
    cred = torch.as_tensor(cred_np)
    dev = torch.device(device) if device is not None else torch.device("cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    M_ui, M_iu = V2.build_message_passing_mats(e, U, I, cred, dev)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0      # the drop-in builder (device graph + scales)
    model = V2.LightGCN(U, I, d, K, M_ui, M_iu).to(dev)   # the reference's module init
    if dense_finals:   # propagate() computes both whole tables at the call
        model.lazy_finals = False
    if pre_ordered:
        assert M_ui.graph.user_csr.cols_by_degree and M_ui.graph.item_csr.cols_by_degree
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0
    t1 = time.perf_counter()
    with torch.no_grad():
        model.propagate()   # first call: operator pair registration + first-layer values
    torch.cuda.synchronize()
    first_call_s = time.perf_counter() - t1
    n_b = warmup + steps
    if batches == "reference":   # in the ids the model was built on
        t2 = time.perf_counter()
        users, pos, neg = (torch.as_tensor(x).to(dev) for x in
                           reference_batches(e, U, I, B, n_b))
        batches_s = time.perf_counter() - t2
    else:
        g = torch.Generator(device=dev).manual_seed(1)
        users = torch.randint(0, U, (n_b, B), device=dev, generator=g)
        pos = torch.randint(0, I, (n_b, B), device=dev, generator=g)
        neg = torch.randint(0, I, (n_b, B), device=dev, generator=g)
        batches_s = 0.0
    it = iter(range(10**9))
    opt = None

    def fwd_bwd():
        k = next(it) % n_b
        uf, itf = model.propagate()
        loss = model.bpr_loss(users[k], pos[k], neg[k], uf, itf, 1e-4)
        opt.zero_grad(set_to_none=True)
        loss.backward()

    def step():
        fwd_bwd()
        opt.step()

    def fwd():   # the step's forward as the reference's loop runs it: tables -> loss
        k = next(it) % n_b
        with torch.no_grad():
            uf, itf = model.propagate()
            model.bpr_loss(users[k], pos[k], neg[k], uf, itf, 1e-4)

    def full_tables():   # every row of both final tables (evaluation's use)
        from bbgr.lazy import resolve
        with torch.no_grad():
            uf, itf = model.propagate()
            resolve(uf)
            resolve(itf)

    res = {}
    for adam in adams:
        if adam in ("bbgr", "bbgr_bwd"):   # bbgr.optim.FusedAdam (bbgr_adam per parameter,
            from bbgr.optim import FusedAdam   # or inside the backward's last products)
            opt = FusedAdam(model.parameters(), lr=1e-3, fuse_backward=adam == "bbgr_bwd")
        else:
            opt = torch.optim.Adam(model.parameters(), lr=1e-3,
                                   **({"fused": True} if adam == "fused" else {"foreach": True}))
        for _ in range(warmup):
            step()
        out = {"config": cfg_name, "adam": adam, "pre_ordered": pre_ordered,
               "items_ordered": items_ordered, "batches": batches,
               "batches_s": batches_s,
               "setup_s": setup_s, "build_s": build_s, "model_init_s": setup_s - build_s,
               "first_call_s": first_call_s, "steps": steps,
               "lazy_finals": bool(model.lazy_finals),
               "step_ms": timed(step, steps), "forward_ms": timed(fwd, steps),
               "full_tables_ms": timed(full_tables, steps),
               "forward_backward_ms": timed(fwd_bwd, steps)}
        fwd_bwd()
        out["adam_ms"] = timed(opt.step, steps)
        out["optimizer"] = ("bbgr.optim.FusedAdam" if adam == "bbgr" else
                            "bbgr.optim.FusedAdam(fuse_backward=True)" if adam == "bbgr_bwd" else
                            f"torch.optim.Adam({adam})")
        res[adam] = out
        opt = None
    del model, M_ui, M_iu, users, pos, neg
    torch.cuda.empty_cache()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--adam", default="foreach", choices=["foreach", "fused", "bbgr", "bbgr_bwd"])
    ap.add_argument("--pre-ordered", action="store_true",
                    help="hand the model an edge list already in descending-degree order")
    ap.add_argument("--items-ordered", action="store_true",
                    help="only the item ids handed over in descending-degree order")
    ap.add_argument("--dense-finals", action="store_true",
                    help="LightGCN.lazy_finals = False: whole final tables at every call")
    ap.add_argument("--batches", default="reference", choices=["reference", "uniform"],
                    help="the reference loop's batches (host sampler, pop-mix) or uniform "
                         "device draws (module docstring)")
    a = ap.parse_args()
    print(json.dumps(run(a.config, steps=a.steps, warmup=a.warmup, adam=a.adam,
                         pre_ordered=a.pre_ordered, items_ordered=a.items_ordered,
                         dense_finals=a.dense_finals, batches=a.batches)),
          flush=True)


if __name__ == "__main__":
    main()
