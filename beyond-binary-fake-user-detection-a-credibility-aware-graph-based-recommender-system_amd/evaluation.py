"""GPU sampled evaluation: drop-in for evaluate_sampled
(Version-2/lighgcn_cu_pop.py:536-650), SURVEY §8(f) row 1.

The reference loops over test users in Python (one torch scoring call and one
device->host copy per user). Here one launch scores every evaluated user's
1 + n_neg candidates (bbgr_eval_sampled), a second computes the metric terms
and a fixed-order reduction sums them; the host reads back a few dozen floats.

Semantics kept: pos uniform from the test row; negatives uniform over items,
rejected if in the test row or the train row, duplicates allowed; ranking
descending by score; P/R/NDCG@K with gt = {pos}; coverage = distinct top-K
items / I; novelty over the top-K (avg log(pop+1), avg -log2((pop+1)/(T+I)));
cred_utility = mean credibility of evaluated users; high/low groups = top /
bottom `pct` of evaluated users by credibility (make_cred_groups :408-426).
Differences (documented, distributional): the RNG is Philox, not numpy's
PCG64 stream; exact score ties rank in candidate order (pos first) where the
reference's quicksort argsort leaves the order unspecified; group membership
at exactly-tied credibility values follows a stable sort.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import call, ld, ptr, stream_handle
from .graph import Csr
from .sampler import nonempty_rows

NOUT = 11   # per K: p, r, ndcg, logpop, selfinfo, high_r, low_r, high_n, low_n, n, covered


def cred_groups(users: torch.Tensor, cred: torch.Tensor, pct: float) -> torch.Tensor:
    """uint8 flags per evaluated user: bit0 = top `pct` by credibility, bit1 =
    bottom `pct` (make_cred_groups, Version-2:408-426; k = max(round(n*pct), 1))."""
    n = users.numel()
    flags = torch.zeros(n, dtype=torch.uint8, device=users.device)
    if n == 0:
        return flags
    k = max(int(round(n * pct)), 1)
    order = torch.sort(cred[users], stable=True).indices
    flags[order[:k]] |= 2
    flags[order[-k:]] |= 1
    return flags


def evaluate_sampled(user_emb: torch.Tensor, item_emb: torch.Tensor, train_csr: Csr,
                     test_csr: Csr, num_items: int, item_pop, total_train_interactions: int,
                     cred, Ks=(10, 20), sampled_negatives: int = 99,
                     cred_group_pct: float = 0.20, seed: int = 42 + 999, counter: int = 0,
                     return_raw: bool = False):
    """Reference-shaped results {K: {...}} for the sampled protocol."""
    _lib.require_gpu(user_emb)
    dev = user_emb.device
    users = nonempty_rows(test_csr)
    if users.numel() == 0:
        raise RuntimeError("No users with test interactions. Check your split or threshold.")
    n = users.numel()
    Ks = tuple(int(k) for k in Ks)
    k_max, n_k, nc = max(Ks), len(Ks), 1 + int(sampled_negatives)
    uf = user_emb.detach().to(torch.float32).contiguous()
    itf = item_emb.detach().to(torch.float32).contiguous()
    pop = torch.as_tensor(np.asarray(item_pop, np.float32) if not isinstance(item_pop, torch.Tensor)
                          else item_pop).to(dev, torch.float32).contiguous()
    cred_t = torch.as_tensor(np.asarray(cred, np.float32) if not isinstance(cred, torch.Tensor)
                             else cred).to(dev, torch.float32).contiguous()
    groups = cred_groups(users, cred_t, cred_group_pct)
    i32 = dict(dtype=torch.int32, device=dev)
    pos_rank = torch.empty(n, **i32)
    topk = torch.empty(n * k_max, **i32)
    cand = torch.empty(n * nc, **i32) if return_raw else None
    fails = torch.zeros(1, **i32)
    stats = torch.empty(n * n_k * 6, dtype=torch.float32, device=dev)
    covered = torch.empty(n_k * num_items, dtype=torch.uint8, device=dev)
    sums = torch.empty(n_k * NOUT, dtype=torch.float32, device=dev)
    a = _lib.EvalArgs()
    a.n_users, a.users = n, ptr(users)
    a.te_indptr, a.te_indices = ptr(test_csr.indptr), ptr(test_csr.indices)
    a.tr_indptr, a.tr_indices = ptr(train_csr.indptr), ptr(train_csr.indices)
    a.uf, a.lduf, a.itf, a.ldif = ptr(uf), ld(uf), ptr(itf), ld(itf)
    a.d, a.n_items, a.n_neg, a.k_max, a.n_k = uf.shape[1], num_items, nc - 1, k_max, n_k
    for q, k in enumerate(Ks):
        a.ks[q] = k
    a.seed, a.counter = int(seed), int(counter)
    a.item_pop, a.self_info_denom = ptr(pop), float(total_train_interactions + num_items)
    a.group = ptr(groups)
    a.pos_rank, a.topk, a.cand_out, a.fail_count = ptr(pos_rank), ptr(topk), ptr(cand), ptr(fails)
    a.stats, a.covered, a.sums = ptr(stats), ptr(covered), ptr(sums)
    call("bbgr_eval_sampled", ctypes.byref(a), stream_handle())
    s = sums.view(n_k, NOUT).double().cpu().numpy()
    cred_utility = float(cred_t[users].double().mean())
    results = {}
    for q, K in enumerate(Ks):
        p, r, nd, lp, si, hr, lr, hn, lnn, ne, cov = s[q]
        ne = max(ne, 1.0)
        results[K] = {
            "precision": p / ne, "recall": r / ne, "ndcg": nd / ne,
            "item_coverage": cov / max(num_items, 1),
            "avg_log_popularity": lp / ne, "avg_self_information": si / ne,
            "cred_utility": cred_utility,
            "high_cred_recall": hr / max(hn, 1.0), "low_cred_recall": lr / max(lnn, 1.0),
            "high_users": int(hn), "low_users": int(lnn),
            "users_eval": int(s[q][9]), "mode": "sampled(1pos+neg)",
            "negatives": int(sampled_negatives),
        }
    if return_raw:
        results["_raw"] = dict(users=users, pos_rank=pos_rank, topk=topk.view(n, k_max),
                               cand=cand.view(n, nc), groups=groups, fails=int(fails.item()))
    return results
