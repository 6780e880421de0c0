"""GPU evaluation: drop-ins for evaluate_sampled (Version-2/lighgcn_cu_pop.py:
536-650) and evaluate_full_ranking (:652-752), SURVEY §8(f) row 1.

The reference loops over test users in Python (one torch scoring call and one
device->host copy per user). Here one launch scores every evaluated user's
1 + n_neg candidates (bbgr_eval_sampled), a second computes the metric terms
and a fixed-order reduction sums them; the host reads back a few dozen floats.

Semantics kept: pos uniform from the test row; negatives uniform over items,
rejected if in the test row or the train row, duplicates allowed; ranking
descending by score; P/R/NDCG@K with gt = {pos}; coverage = distinct top-K
items / I; novelty over the top-K (avg log(pop+1), avg -log2((pop+1)/(T+I)));
cred_utility = mean credibility of evaluated users; high/low groups = top /
bottom `pct` of evaluated users by credibility (make_cred_groups :405-422).
The reference-signature wrappers (evaluate_sampled_reference, exported by
each drop-in module as `evaluate_sampled`) draw the candidates from the
reference's own stream: np.random.default_rng(seed + 999), the positive and
the rejection-sampled negatives per user in order (bbgr_eval_draw_candidates,
numpy's PCG64 + bounded-integer path restated in host C, bit for bit, the
Generator left in numpy's end state), and form the credibility groups with
the reference's np.argsort (make_cred_groups). The kernel then scores the
supplied candidates. The native evaluate_sampled draws on the device (Philox,
a different stream with the same law) unless given candidates. Exact score
ties rank in candidate order (pos first) where the reference's quicksort
argsort leaves the order unspecified; with distinct items they need equal
dot products.
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


def make_cred_groups(users: np.ndarray, cred: np.ndarray, pct: float):
    """The reference's make_cred_groups (Version-2/lighgcn_cu_pop.py:408-426):
    (high, low) user arrays, the top / bottom `pct` of `users` by credibility
    through numpy's default argsort, so tied credibilities split exactly as
    the reference splits them."""
    if users.size == 0:
        return np.array([], dtype=np.int64), np.array([], dtype=np.int64)
    c = cred[users]
    n = users.size
    k = max(int(round(n * pct)), 1)
    order = np.argsort(c)  # ascending (the reference's call: quicksort)
    return users[order[-k:]].astype(np.int64), users[order[:k]].astype(np.int64)


def cred_group_flags(users: np.ndarray, cred: np.ndarray, pct: float) -> np.ndarray:
    """make_cred_groups as uint8 flags per evaluated user (bit0 high, bit1 low)."""
    flags = np.zeros(users.size, dtype=np.uint8)
    if users.size == 0:
        return flags
    k = max(int(round(users.size * pct)), 1)
    order = np.argsort(cred[users])
    flags[order[:k]] |= 2
    flags[order[-k:]] |= 1
    return flags


def pcg64_state(rng: np.random.Generator) -> "_lib.Pcg64State":
    """A numpy Generator's PCG64 state as bbgr_pcg64."""
    st = rng.bit_generator.state
    if st["bit_generator"] != "PCG64":
        raise ValueError(f"the reference's stream is PCG64; got {st['bit_generator']}")
    s, inc = int(st["state"]["state"]), int(st["state"]["inc"])
    m = (1 << 64) - 1
    return _lib.Pcg64State(s >> 64, s & m, inc >> 64, inc & m, int(st["has_uint32"]),
                           int(st["uinteger"]))


def set_pcg64_state(rng: np.random.Generator, c) -> None:
    """Write a bbgr_pcg64 back into the Generator (numpy's own state dict)."""
    st = rng.bit_generator.state
    st["state"]["state"] = (int(c.state_hi) << 64) | int(c.state_lo)
    st["has_uint32"], st["uinteger"] = int(c.has_uint32), int(c.uinteger)
    rng.bit_generator.state = st


def draw_candidates(rng: np.random.Generator, users: np.ndarray, train_csr, test_csr,
                    num_items: int, n_neg: int) -> np.ndarray:
    """int32 [n_users, 1 + n_neg]: the positive and negatives evaluate_sampled
    (Version-2/lighgcn_cu_pop.py:575-589) draws for each user in order from
    `rng`, which is advanced exactly as the reference's loop advances it
    (bbgr_eval_draw_candidates; host code, no GPU)."""
    users = np.ascontiguousarray(users, dtype=np.int64)
    tr_p, tr_i = (np.ascontiguousarray(x, dtype=np.int64) for x in train_csr)
    te_p, te_i = (np.ascontiguousarray(x, dtype=np.int64) for x in test_csr)
    cand = np.empty((users.size, 1 + int(n_neg)), dtype=np.int32)
    c = pcg64_state(rng)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)   # noqa: E731
    call("bbgr_eval_draw_candidates", ctypes.byref(c), users.size, p(users), p(te_p), p(te_i),
         p(tr_p), p(tr_i), int(num_items), int(n_neg), p(cand))
    set_pcg64_state(rng, c)
    return cand


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


def _tables(user_emb, item_emb, item_pop, cred, dev):
    uf = user_emb.detach().to(torch.float32).contiguous()
    itf = item_emb.detach().to(torch.float32).contiguous()
    pop = torch.as_tensor(np.asarray(item_pop, np.float32) if not isinstance(item_pop, torch.Tensor)
                          else item_pop).to(dev, torch.float32).contiguous()
    cred_t = torch.as_tensor(np.asarray(cred, np.float32) if not isinstance(cred, torch.Tensor)
                             else cred).to(dev, torch.float32).contiguous()
    return uf, itf, pop, cred_t


def _args(users, train_csr, test_csr, uf, itf, num_items, Ks, pop, total_train, groups, sums):
    a = _lib.EvalArgs()
    a.n_users, a.users = users.numel(), ptr(users)
    a.te_indptr, a.te_indices = ptr(test_csr.indptr), ptr(test_csr.indices)
    a.tr_indptr, a.tr_indices = ptr(train_csr.indptr), ptr(train_csr.indices)
    a.uf, a.lduf, a.itf, a.ldif = ptr(uf), ld(uf), ptr(itf), ld(itf)
    a.d, a.n_items, a.k_max, a.n_k = uf.shape[1], num_items, max(Ks), len(Ks)
    for q, k in enumerate(Ks):
        a.ks[q] = k
    a.item_pop, a.self_info_denom = ptr(pop), float(total_train + num_items)
    a.group, a.sums = ptr(groups), ptr(sums)
    return a


def _run(fn, a, dev):
    n = ctypes.c_size_t(0)
    call(fn, ctypes.byref(a), None, ctypes.byref(n), stream_handle())
    ws = torch.empty(max(n.value, 1), dtype=torch.uint8, device=dev)
    call(fn, ctypes.byref(a), ptr(ws), ctypes.byref(n), stream_handle())
    return ws


def _results(sums, Ks, num_items, cred_utility, mode, extra):
    s = sums.view(len(Ks), NOUT).cpu().numpy()
    results = {}
    for q, K in enumerate(Ks):
        p, r, nd, lp, si, hr, lr, hn, lnn, ne, cov = s[q]
        nd_ = max(ne, 1.0)
        results[K] = {
            "precision": p / nd_, "recall": r / nd_, "ndcg": nd / nd_,
            "item_coverage": cov / max(num_items, 1),
            "avg_log_popularity": lp / nd_, "avg_self_information": si / nd_,
            "cred_utility": cred_utility,
            "high_cred_recall": hr / max(hn, 1.0), "low_cred_recall": lr / max(lnn, 1.0),
            "high_users": int(hn), "low_users": int(lnn),
            "users_eval": int(ne), "mode": mode, **extra,
        }
    return results


def _eval_users(test_csr):
    users = nonempty_rows(test_csr)
    if users.numel() == 0:
        raise RuntimeError("No users with test interactions. Check your split or threshold.")
    return users


def evaluate_sampled(user_emb: torch.Tensor, item_emb: torch.Tensor, train_csr: Csr,
                     test_csr: Csr, num_items: int, item_pop, total_train_interactions: int,
                     cred, Ks=(10, 20), sampled_negatives: int = 99,
                     cred_group_pct: float = 0.20, seed: int = 42 + 999, counter: int = 0,
                     return_raw: bool = False, cand=None, users=None, groups=None,
                     cred_utility=None):
    """Reference-shaped results {K: {...}} for the sampled protocol.

    cand (int32 [n_users, 1 + sampled_negatives], host or device): score these
    candidates (c = 0 the positive) instead of drawing them on the device;
    users / groups / cred_utility: the evaluated users (int64, ascending),
    their uint8 group flags and the credibility mean, when the caller formed
    them (the reference-signature wrapper does, on the host)."""
    _lib.require_gpu(user_emb)
    dev = user_emb.device
    users = _eval_users(test_csr) if users is None else users.to(dev, torch.int64)
    n = users.numel()
    Ks = tuple(int(k) for k in Ks)
    nc = 1 + int(sampled_negatives)
    uf, itf, pop, cred_t = _tables(user_emb, item_emb, item_pop, cred, dev)
    groups = (cred_groups(users, cred_t, cred_group_pct) if groups is None
              else torch.as_tensor(groups).to(dev, torch.uint8))
    cand_in = None
    if cand is not None:
        cand_in = torch.as_tensor(cand).to(dev, torch.int32).contiguous()
        if cand_in.numel() != n * nc:
            raise ValueError(f"cand: {n} users x {nc} candidates expected")
    i32 = dict(dtype=torch.int32, device=dev)
    pos_rank = torch.empty(n, **i32)
    topk = torch.empty(n * max(Ks), **i32)
    cand = torch.empty(n * nc, **i32) if return_raw else None
    fails = torch.zeros(1, **i32)
    sums = torch.empty(len(Ks) * NOUT, dtype=torch.float64, device=dev)
    a = _args(users, train_csr, test_csr, uf, itf, num_items, Ks, pop,
              total_train_interactions, groups, sums)
    a.n_neg, a.seed, a.counter = nc - 1, int(seed), int(counter)
    a.pos_rank, a.topk, a.cand_out, a.fail_count = ptr(pos_rank), ptr(topk), ptr(cand), ptr(fails)
    a.cand_in = ptr(cand_in)
    _run("bbgr_eval_sampled", a, dev)
    cu = float(cred_t[users].double().mean()) if cred_utility is None else cred_utility
    results = _results(sums, Ks, num_items, cu, "sampled(1pos+neg)",
                       {"negatives": int(sampled_negatives)})
    if return_raw:
        results["_raw"] = dict(users=users, pos_rank=pos_rank, topk=topk.view(n, max(Ks)),
                               cand=cand.view(n, nc), groups=groups, fails=int(fails.item()))
    return results


def evaluate_full(user_emb: torch.Tensor, item_emb: torch.Tensor, train_csr: Csr,
                  test_csr: Csr, num_items: int, item_pop, total_train_interactions: int,
                  cred, Ks=(10, 20), cred_group_pct: float = 0.20, return_raw: bool = False,
                  users=None, groups=None, cred_utility=None):
    """Drop-in for evaluate_full_ranking (Version-2/lighgcn_cu_pop.py:652-752).

    One bbgr_eval_full call scores every (evaluated user, item) pair with fp32
    MFMA, masks train items to -1e9 and keeps the top-max(Ks) per user in
    registers (no U x I score matrix is ever written), then reduces the
    metrics. Ranking ties (unspecified in the reference's torch.argsort) go
    to the lower item id."""
    _lib.require_gpu(user_emb)
    dev = user_emb.device
    users = _eval_users(test_csr) if users is None else users.to(dev, torch.int64)
    n = users.numel()
    Ks = tuple(int(k) for k in Ks)
    uf, itf, pop, cred_t = _tables(user_emb, item_emb, item_pop, cred, dev)
    groups = (cred_groups(users, cred_t, cred_group_pct) if groups is None
              else torch.as_tensor(groups).to(dev, torch.uint8))
    topk = torch.empty(n * max(Ks), dtype=torch.int32, device=dev)
    topk_score = torch.empty(n * max(Ks), dtype=torch.float32, device=dev) if return_raw else None
    sums = torch.empty(len(Ks) * NOUT, dtype=torch.float64, device=dev)
    a = _args(users, train_csr, test_csr, uf, itf, num_items, Ks, pop,
              total_train_interactions, groups, sums)
    a.topk, a.topk_score = ptr(topk), ptr(topk_score)
    _run("bbgr_eval_full", a, dev)
    cu = float(cred_t[users].double().mean()) if cred_utility is None else cred_utility
    results = _results(sums, Ks, num_items, cu, "full", {})
    if return_raw:
        results["_raw"] = dict(users=users, topk=topk.view(n, max(Ks)),
                               topk_score=topk_score.view(n, max(Ks)), groups=groups)
    return results


# -- the reference scripts' evaluate_* signatures ------------------------------
# Version-2/lighgcn_cu_pop.py:536-752 take (model, train_csr, test_csr,
# num_items, device, item_pop, total_train_interactions, cred_np) with host
# (indptr, indices) CSRs from edges_to_user_csr and read cfg.Ks /
# cfg.sampled_negatives / cfg.cred_group_pct / cfg.seed; the older scripts
# (version_1/*.py:486-610, lightgcn_cu.py:488-560, lightgcn.py:398-520) take
# the first five only and return precision / recall / ndcg per K. The
# wrappers below keep those signatures (the cfg fields as keyword arguments
# with the reference's defaults) and return the same dictionaries. Sampled
# candidates are drawn on the device (Philox), not from the host Generator.
_V1_KEYS = ("precision", "recall", "ndcg", "users_eval", "mode")


def csr_from_host(csr, n_cols: int, device) -> Csr:
    """A host (indptr, indices) CSR (edges_to_user_csr) as a device Csr."""
    indptr, indices = csr
    indptr = np.asarray(indptr, dtype=np.int64)
    n_rows = indptr.size - 1
    rows = np.repeat(np.arange(n_rows, dtype=np.int32), np.diff(indptr))
    return Csr(rows, np.asarray(indices).astype(np.int32), n_rows, n_cols, device)


def _model_tables(model, device):
    """The final tables as each reference evaluate_* reads them:
    final_embeddings() (CredLightGCN, lightgcn_cu.py:492) or get_user_item_emb()."""
    with torch.no_grad():
        if hasattr(model, "final_embeddings"):
            ue, ie = model.final_embeddings()
        else:
            ue, ie = model.get_user_item_emb()
        dev = torch.device(device)
        return ue.to(dev), ie.to(dev)


def _host_defaults(train_csr, num_items, n_users):
    """item_pop / total interactions / credibility for the five-argument
    scripts, whose results carry none of the metrics they feed."""
    pop = np.bincount(np.asarray(train_csr[1], np.int64), minlength=num_items)
    return pop.astype(np.float32), int(pop.sum()), np.ones(n_users, np.float32)


def _host_users(test_csr, cred_np, pct):
    """The evaluated users, their group flags and the credibility mean exactly
    as the reference forms them (Version-2:556-568, :595, :634): users =
    np.where(test row lengths > 0), make_cred_groups' np.argsort, and
    cred_sum accumulated user by user in double (np.add.accumulate is that
    sequential sum)."""
    indptr_te = np.asarray(test_csr[0])
    users = np.where((indptr_te[1:] - indptr_te[:-1]) > 0)[0].astype(np.int64)
    if len(users) == 0:
        raise RuntimeError("No users with test interactions. Check your split or threshold.")
    cred = np.asarray(cred_np)
    flags = cred_group_flags(users, cred, pct)
    cred_sum = float(np.add.accumulate(cred[users].astype(np.float64))[-1])
    return users, flags, cred_sum / users.size


def evaluate_sampled_reference(model, train_csr, test_csr, num_items: int, device,
                               item_pop=None, total_train_interactions=None, cred_np=None, *,
                               Ks=(10, 20), sampled_negatives: int = 99,
                               cred_group_pct: float = 0.20, seed: int = 42,
                               candidates: str = "numpy", return_raw: bool = False):
    """evaluate_sampled with the reference scripts' signature (see above).
    candidates="numpy" (default): the reference's stream, bit for bit;
    "philox": drawn on the device (same law, another stream)."""
    ue, ie = _model_tables(model, device)
    v1 = item_pop is None
    if v1:
        item_pop, total_train_interactions, cred_np = _host_defaults(train_csr, num_items,
                                                                     ue.shape[0])
    tr = csr_from_host(train_csr, num_items, ue.device)
    te = csr_from_host(test_csr, num_items, ue.device)
    if candidates == "philox":
        res = evaluate_sampled(ue, ie, tr, te, num_items, item_pop, total_train_interactions,
                               cred_np, Ks=Ks, sampled_negatives=sampled_negatives,
                               cred_group_pct=cred_group_pct, seed=seed + 999,
                               return_raw=return_raw)
    elif candidates == "numpy":
        users, flags, cred_utility = _host_users(test_csr, cred_np, cred_group_pct)
        rng = np.random.default_rng(seed + 999)
        cand = draw_candidates(rng, users, train_csr, test_csr, num_items, sampled_negatives)
        res = evaluate_sampled(ue, ie, tr, te, num_items, item_pop, total_train_interactions,
                               cred_np, Ks=Ks, sampled_negatives=sampled_negatives,
                               cred_group_pct=cred_group_pct, return_raw=return_raw,
                               cand=torch.from_numpy(cand), users=torch.from_numpy(users),
                               groups=torch.from_numpy(flags), cred_utility=cred_utility)
        if return_raw:
            res["_raw"]["rng_state"] = rng.bit_generator.state
    else:
        raise ValueError(f"candidates must be 'numpy' or 'philox', got {candidates!r}")
    if v1:
        raw = res.pop("_raw", None)
        res = {K: {**{k: r[k] for k in _V1_KEYS}, "negatives": r["negatives"]}
               for K, r in res.items()}
        if raw is not None:
            res["_raw"] = raw
    return res


def evaluate_full_ranking_reference(model, train_csr, test_csr, num_items: int, device,
                                    item_pop=None, total_train_interactions=None, cred_np=None,
                                    *, Ks=(10, 20), cred_group_pct: float = 0.20):
    """evaluate_full_ranking with the reference scripts' signature (see above)."""
    ue, ie = _model_tables(model, device)
    v1 = item_pop is None
    if v1:
        item_pop, total_train_interactions, cred_np = _host_defaults(train_csr, num_items,
                                                                     ue.shape[0])
    tr = csr_from_host(train_csr, num_items, ue.device)
    te = csr_from_host(test_csr, num_items, ue.device)
    users, flags, cred_utility = _host_users(test_csr, cred_np, cred_group_pct)
    res = evaluate_full(ue, ie, tr, te, num_items, item_pop, total_train_interactions, cred_np,
                        Ks=Ks, cred_group_pct=cred_group_pct, users=torch.from_numpy(users),
                        groups=torch.from_numpy(flags), cred_utility=cred_utility)
    if v1:
        res = {K: {k: r[k] for k in _V1_KEYS} for K, r in res.items()}
    return res
