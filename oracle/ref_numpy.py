"""ORACLE (test infrastructure only): float64 numpy/scipy restatement of the
reference hot path. Each function cites the reference lines it follows
(paths relative to the reference repository root).

Operator VALUES are computed in float32 exactly as the reference's numpy code
does (they are fp32 in the reference); propagation, loss and gradients are
then evaluated in float64 — the "float64 truth" of the parity criterion.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


# ---------------------------------------------------------------------------
# CSR helpers and samplers (Version-2/lighgcn_cu_pop.py:309-376)
# ---------------------------------------------------------------------------
def edges_to_user_csr(edges_2xE: np.ndarray, num_users: int):
    """Version-2/lighgcn_cu_pop.py:309-327 (vectorised: stable sort by
    (user, item) == mergesort by user then per-row np.sort)."""
    u = edges_2xE[0].astype(np.int64)
    it = edges_2xE[1].astype(np.int64)
    counts = np.bincount(u, minlength=num_users)
    indptr = np.zeros(num_users + 1, dtype=np.int64)
    indptr[1:] = np.cumsum(counts)
    if it.size == 0:
        return indptr, it.copy()
    # rows by user, items ascending inside a row: the sorted (user, item) keys
    # (equal keys are equal pairs, so a plain sort is the stable one)
    m = int(it.max()) + 1
    keys = np.sort(u * m + it)
    return indptr, keys % m


def user_has_item(indptr, indices, user: int, item: int) -> bool:
    """Version-2/lighgcn_cu_pop.py:330-336."""
    start, end = indptr[user], indptr[user + 1]
    if start == end:
        return False
    arr = indices[start:end]
    j = np.searchsorted(arr, item)
    return bool(j < (end - start) and arr[j] == item)


def sample_pos_item(indptr, indices, user: int, rng: np.random.Generator):
    """Version-2/lighgcn_cu_pop.py:339-343."""
    start, end = indptr[user], indptr[user + 1]
    if start == end:
        return None
    return int(indices[rng.integers(start, end)])


def sample_neg_item(indptr, indices, user: int, num_items: int, rng: np.random.Generator):
    """lightgcn.py:296-300 (uniform)."""
    while True:
        j = int(rng.integers(0, num_items))
        if not user_has_item(indptr, indices, user, j):
            return j


def sample_neg_item_popmix(indptr, indices, user: int, num_items: int,
                           rng: np.random.Generator, pop_prob: np.ndarray,
                           mix_pop: float, max_tries: int):
    """Version-2/lighgcn_cu_pop.py:349-376."""
    for _ in range(max_tries):
        if rng.random() < mix_pop:
            j = int(rng.choice(num_items, p=pop_prob))
        else:
            j = int(rng.integers(0, num_items))
        if not user_has_item(indptr, indices, user, j):
            return j
    while True:
        j = int(rng.integers(0, num_items))
        if not user_has_item(indptr, indices, user, j):
            return j


def pop_prob(train_edges_2xE: np.ndarray, num_items: int, gamma: float = 0.75):
    """Version-2/lighgcn_cu_pop.py:805-810."""
    item_deg = np.bincount(train_edges_2xE[1].astype(np.int64),
                           minlength=num_items).astype(np.float64)
    pop = np.power(item_deg + 1.0, gamma)
    return (pop / (pop.sum() + 1e-12)).astype(np.float64)


def sample_batch_reference_style(indptr, indices, users, num_items, rng, pop_prob_,
                                 mix_pop=0.7, max_tries=50):
    """The per-user host loop of Version-2/lighgcn_cu_pop.py:835-849."""
    used, pos, neg = [], [], []
    for u in users:
        p = sample_pos_item(indptr, indices, int(u), rng)
        if p is None:
            continue
        n = sample_neg_item_popmix(indptr, indices, int(u), num_items, rng,
                                   pop_prob=pop_prob_, mix_pop=mix_pop, max_tries=max_tries)
        used.append(int(u))
        pos.append(p)
        neg.append(n)
    return np.array(used), np.array(pos), np.array(neg)


def sample_batch_uniform_reference_style(indptr, indices, users, num_items, rng):
    """The per-user host loop of lightgcn_cu.py:611-621 (== lightgcn.py:565-575):
    a uniform positive from the row, a uniform negative rejected while the user
    has it (sample_neg_item)."""
    used, pos, neg = [], [], []
    for u in users:
        p = sample_pos_item(indptr, indices, int(u), rng)
        if p is None:
            continue
        used.append(int(u))
        pos.append(p)
        neg.append(sample_neg_item(indptr, indices, int(u), num_items, rng))
    return np.array(used), np.array(pos), np.array(neg)


# ---------------------------------------------------------------------------
# Operator values (fp32, as the reference computes them)
# ---------------------------------------------------------------------------
def degrees(edges_2xE, num_users, num_items):
    """fp32 (deg_u, deg_i) as the reference builders compute them: np.bincount
    of the edge list -> float32 (Version-2/lighgcn_cu_pop.py:434-435,
    lightgcn_cu.py:383-384). Duplicate pairs count with their multiplicity."""
    deg_u = np.bincount(edges_2xE[0].astype(np.int64), minlength=num_users).astype(np.float32)
    deg_i = np.bincount(edges_2xE[1].astype(np.int64), minlength=num_items).astype(np.float32)
    return deg_u, deg_i


def edge_weights(kind, u, i, deg_u, deg_i, cred_u=None):
    """Per-edge fp32 operator values of the edges (u[e], i[e]) given the graph's
    fp32 degrees — the reference's weight expressions evaluated on any subset
    of the edges (the full-size parity tests check sampled rows only).
    Returns (w_user_from_item, w_item_from_user):
      "gs" / "method_a": Version-2/lighgcn_cu_pop.py:436-450 (M_ui[u,i] = w_base,
          M_iu[i,u] = c_u * w_base); method_a also x alpha_i,
          version_1/lightgcn_cu_pop_long_tail_exposure.py:379-392
      "j": lightgcn_cu.py:385-397 (item<-user c_u/denom, user<-item 1/denom)
      "sym": lightgcn.py:365-372 (deg^-1/2 on both ends, inf -> 0; one
          entry per edge, so a duplicate pair sums to v * dinv_r * dinv_c)."""
    u = np.asarray(u, np.int64)
    i = np.asarray(i, np.int64)
    c = None if cred_u is None else np.asarray(cred_u, np.float32)
    if kind in ("gs", "method_a"):
        inv_sqrt_u = 1.0 / np.sqrt(np.maximum(deg_u, 1.0))
        inv_sqrt_i = 1.0 / np.sqrt(np.maximum(deg_i, 1.0))
        w_base = inv_sqrt_u[u] * inv_sqrt_i[i]
        if kind == "method_a":
            alpha_i = (1.0 / np.log1p(np.maximum(deg_i, 1.0))).astype(np.float32)
            w_base = w_base * alpha_i[i]
        w_cred = w_base if c is None else c[u] * w_base
        return w_base.astype(np.float32), w_cred.astype(np.float32)
    if kind == "j":
        denom = np.sqrt(np.maximum(deg_u[u] * deg_i[i], 1e-12)).astype(np.float32)
        w_iu = (1.0 / denom).astype(np.float32)
        w_ui = (np.float32(1.0) / denom if c is None else c[u] / denom).astype(np.float32)
        return w_iu, w_ui
    if kind == "sym":
        with np.errstate(divide="ignore"):
            du = np.power(deg_u, np.float32(-0.5)).astype(np.float32)
            di = np.power(deg_i, np.float32(-0.5)).astype(np.float32)
        du[np.isinf(du)] = 0.0
        di[np.isinf(di)] = 0.0
        w = (np.float32(1.0) * du[u] * di[i]).astype(np.float32)
        return w, w
    raise ValueError(f"unknown operator kind {kind!r}")


def rows_product(sel_rows, rows, cols, w, x_cols):
    """float64 y[sel_rows[k]] = sum over the edges e of that row of
    w[e] * x_cols[e] — one sparse product evaluated on a subset of its output
    rows (torch.sparse.mm of Version-2:483-484 / lightgcn_cu.py:431,434 /
    lightgcn.py:323 restricted to those rows). rows[e] must be in sel_rows;
    x_cols[e] is the source row of edge e (any float dtype). Sums in float64
    (segment sums over the edges grouped by output row)."""
    sel_rows = np.asarray(sel_rows, np.int64)
    x_cols = np.asarray(x_cols)
    srt = np.argsort(sel_rows, kind="stable")
    slot = srt[np.searchsorted(sel_rows[srt], np.asarray(rows, np.int64))]
    out = np.zeros((sel_rows.size, x_cols.shape[1]), np.float64)
    if slot.size == 0:
        return out
    o = np.argsort(slot, kind="stable")
    contrib = np.asarray(w, np.float64)[o, None] * x_cols[o].astype(np.float64)
    starts = np.searchsorted(slot[o], np.arange(sel_rows.size))
    ends = np.append(starts[1:], slot.size)
    nz = ends > starts
    out[nz] = np.add.reduceat(contrib, starts[nz], axis=0)
    return out


def gs_values(edges_2xE, num_users, num_items, cred_u=None, method_a=False):
    """Version-2/lighgcn_cu_pop.py:430-450 (method_a: version_1/
    lightgcn_cu_pop_long_tail_exposure.py:379-392).
    Returns (u, i, w_ui, w_iu): M_ui[u,i] += w_ui, M_iu[i,u] += w_iu."""
    u = edges_2xE[0].astype(np.int64)
    i = edges_2xE[1].astype(np.int64)
    deg_u, deg_i = degrees(edges_2xE, num_users, num_items)
    w_base, w_cred = edge_weights("method_a" if method_a else "gs", u, i, deg_u, deg_i,
                                  np.ones(num_users, np.float32) if cred_u is None else cred_u)
    return u, i, w_base, w_cred


def j_values(edges_2xE, num_users, num_items, cred_u=None):
    """lightgcn_cu.py:383-397. Returns (u, i, w_item_from_user, w_user_from_item, deg_i):
    M_ui[i,u] (item<-user) = c_u/denom, M_iu[u,i] (user<-item) = 1/denom."""
    u = edges_2xE[0].astype(np.int64)
    i = edges_2xE[1].astype(np.int64)
    deg_u, deg_i = degrees(edges_2xE, num_users, num_items)
    w_iu, w_ui = edge_weights("j", u, i, deg_u, deg_i,
                              np.ones(num_users, np.float32) if cred_u is None else cred_u)
    return u, i, w_ui, w_iu, deg_i


def sym_values(edges_2xE, num_users, num_items):
    """lightgcn.py:352-372 after coalesce: returns scipy CSR [N,N] float64 of
    the fp32 values v * dinv[r] * dinv[c] with v = multiplicity."""
    u = edges_2xE[0].astype(np.int64)
    it = edges_2xE[1].astype(np.int64) + num_users
    N = num_users + num_items
    row = np.concatenate([u, it])
    col = np.concatenate([it, u])
    A = sp.coo_matrix((np.ones(row.size, np.float32), (row, col)), shape=(N, N)).tocsr()
    A.sum_duplicates()
    deg = np.asarray(A.sum(axis=1)).ravel().astype(np.float32)
    with np.errstate(divide="ignore"):
        dinv = np.power(deg, np.float32(-0.5)).astype(np.float32)
    dinv[np.isinf(dinv)] = 0.0
    coo = A.tocoo()
    v = (coo.data.astype(np.float32) * dinv[coo.row] * dinv[coo.col]).astype(np.float32)
    return sp.csr_matrix((v.astype(np.float64), (coo.row, coo.col)), shape=(N, N))


def csr64(rows, cols, vals, shape) -> sp.csr_matrix:
    """Coalesced (duplicates summed) float64 matrix of fp32 values."""
    m = sp.coo_matrix((np.asarray(vals, np.float64), (rows, cols)), shape=shape).tocsr()
    m.sum_duplicates()
    return m


def gs_mats(edges_2xE, U, I, cred_u=None, method_a=False):
    u, i, w_ui, w_iu = gs_values(edges_2xE, U, I, cred_u, method_a)
    return csr64(u, i, w_ui, (U, I)), csr64(i, u, w_iu, (I, U))   # M_ui, M_iu


def j_mats(edges_2xE, U, I, cred_u=None):
    u, i, w_ui, w_iu, deg_i = j_values(edges_2xE, U, I, cred_u)
    return csr64(i, u, w_ui, (I, U)), csr64(u, i, w_iu, (U, I)), deg_i  # M_ui[I,U], M_iu[U,I]


# ---------------------------------------------------------------------------
# Propagation (float64)
# ---------------------------------------------------------------------------
def propagate_gs(M_ui, M_iu, u0, i0, K):
    """Version-2/lighgcn_cu_pop.py:472-490. Returns (u_final, i_final, us, is_)."""
    u, i = np.asarray(u0, np.float64), np.asarray(i0, np.float64)
    us, is_ = [u], [i]
    for _ in range(K):
        i = M_iu @ u
        u = M_ui @ i
        us.append(u)
        is_.append(i)
    return np.mean(us, 0), np.mean(is_, 0), us, is_


def propagate_j(M_item_from_user, M_user_from_item, u0, i0, K):
    """lightgcn_cu.py:420-448 (M_ui [I,U] item<-user, M_iu [U,I]; u' uses is_[-1])."""
    us = [np.asarray(u0, np.float64)]
    is_ = [np.asarray(i0, np.float64)]
    for _ in range(K):
        e_i = M_item_from_user @ us[-1]
        e_u = M_user_from_item @ is_[-1]
        us.append(e_u)
        is_.append(e_i)
    return np.mean(us, 0), np.mean(is_, 0), us, is_


def propagate_sym(A, x0, K):
    """lightgcn.py:318-325."""
    x = np.asarray(x0, np.float64)
    xs = [x]
    for _ in range(K):
        x = A @ x
        xs.append(x)
    return np.mean(xs, 0), xs


def backward_gs(M_ui, M_iu, gU, gI, K):
    """Adjoint of propagate_gs: grads of (u0, i0) from dL/du_final, dL/di_final."""
    gl = 1.0 / (K + 1)
    gU, gI = np.asarray(gU, np.float64) * gl, np.asarray(gI, np.float64) * gl
    Gu = gU.copy()
    for _ in range(K):
        Gi = gI + M_ui.T @ Gu
        Gu = gU + M_iu.T @ Gi
    return Gu, gI.copy()


def backward_j(M_item_from_user, M_user_from_item, gU, gI, K):
    gl = 1.0 / (K + 1)
    gU, gI = np.asarray(gU, np.float64) * gl, np.asarray(gI, np.float64) * gl
    Gu, Gi = gU.copy(), gI.copy()
    for _ in range(K):
        Gu, Gi = gU + M_item_from_user.T @ Gi, gI + M_user_from_item.T @ Gu
    return Gu, Gi


def backward_sym(A, g, K):
    gl = 1.0 / (K + 1)
    g = np.asarray(g, np.float64) * gl
    G = g.copy()
    for _ in range(K):
        G = g + A.T @ G
    return G


# ---------------------------------------------------------------------------
# BPR (+reg, +fair) and its gradients (float64)
# ---------------------------------------------------------------------------
def _sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def bpr_loss(uf, itf, ue, ie, users, pos, neg, reg, pop=None, lambda_fair=0.0):
    """Version-2/lighgcn_cu_pop.py:495-508 (+ lightgcn_cu.py:641-648 fair term).
    Returns (loss, grads dict with dense g_uf, g_if, g_ue, g_ie)."""
    uf, itf = np.asarray(uf, np.float64), np.asarray(itf, np.float64)
    ue, ie = np.asarray(ue, np.float64), np.asarray(ie, np.float64)
    users, pos, neg = (np.asarray(a, np.int64) for a in (users, pos, neg))
    B = users.size
    u, p, n = uf[users], itf[pos], itf[neg]
    sp_, sn = (u * p).sum(1), (u * n).sum(1)
    x = sp_ - sn
    sig = _sigmoid(x)
    loss_bpr = -np.log(sig + 1e-12).mean()
    r = ((ue[users] ** 2).sum(1) + (ie[pos] ** 2).sum(1) + (ie[neg] ** 2).sum(1)).mean()
    fair = 0.0 if pop is None else (np.asarray(pop, np.float64)[pos] * sp_).mean()
    loss = loss_bpr + reg * r + lambda_fair * fair
    gx = -(sig * (1.0 - sig)) / (sig + 1e-12) / B
    gpos = gx + (0.0 if pop is None else lambda_fair * np.asarray(pop, np.float64)[pos] / B)
    gneg = -gx
    g_uf = np.zeros_like(uf)
    g_if = np.zeros_like(itf)
    np.add.at(g_uf, users, gpos[:, None] * p + gneg[:, None] * n)
    np.add.at(g_if, pos, gpos[:, None] * u)
    np.add.at(g_if, neg, gneg[:, None] * u)
    g_ue = np.zeros_like(ue)
    g_ie = np.zeros_like(ie)
    np.add.at(g_ue, users, 2.0 * reg / B * ue[users])
    np.add.at(g_ie, pos, 2.0 * reg / B * ie[pos])
    np.add.at(g_ie, neg, 2.0 * reg / B * ie[neg])
    return float(loss), dict(g_uf=g_uf, g_if=g_if, g_ue=g_ue, g_ie=g_ie,
                             parts=np.stack([-np.log(sig + 1e-12),
                                             (ue[users] ** 2).sum(1) + (ie[pos] ** 2).sum(1)
                                             + (ie[neg] ** 2).sum(1),
                                             np.zeros(B) if pop is None else
                                             np.asarray(pop, np.float64)[pos] * sp_], 1))


def adam_step(p, g, m, v, step, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8):
    """torch.optim.Adam (amsgrad=False, weight_decay=0) in float64."""
    p, g, m, v = (np.asarray(a, np.float64).copy() for a in (p, g, m, v))
    m = m + (1 - beta1) * (g - m)
    v = beta2 * v + (1 - beta2) * g * g
    bc1 = 1 - beta1 ** step
    bc2s = np.sqrt(1 - beta2 ** step)
    p = p - (lr / bc1) * m / (np.sqrt(v) / bc2s + eps)
    return p, m, v


def xavier_uniform(rows, cols, rng):
    """torch.nn.init.xavier_uniform_ bound for an [rows, cols] weight."""
    a = np.sqrt(6.0 / (rows + cols))
    return rng.uniform(-a, a, size=(rows, cols)).astype(np.float32)


# ---------------------------------------------------------------------------
# Sampled evaluation given the candidates (Version-2/lighgcn_cu_pop.py:514-650)
# ---------------------------------------------------------------------------
def metrics_at_k(ranked_items, gt_set, K):
    """Version-2/lighgcn_cu_pop.py:514-531."""
    import math
    topk = ranked_items[:K]
    hits = [1 if x in gt_set else 0 for x in topk]
    hit_count = sum(hits)
    precision = hit_count / K
    recall = hit_count / max(len(gt_set), 1)
    dcg = sum(1.0 / math.log2(idx + 2) for idx, h in enumerate(hits) if h)
    ideal = min(len(gt_set), K)
    idcg = sum(1.0 / math.log2(i + 2) for i in range(ideal))
    return precision, recall, (dcg / idcg) if idcg > 0 else 0.0


def evaluate_sampled_given(users, cands, uf, itf, item_pop, total_train, num_items, cred,
                           groups_high, groups_low, Ks=(10, 20)):
    """The reference's per-user loop (Version-2:574-650) on FIXED candidates
    (cands[b] = [pos, neg_1..]), float64 scores, ranking by descending score
    with ties in candidate order."""
    uf, itf = np.asarray(uf, np.float64), np.asarray(itf, np.float64)
    item_pop = np.asarray(item_pop, np.float64)
    sums = {K: dict(p=0.0, r=0.0, n=0.0, lp=0.0, si=0.0) for K in Ks}
    rec = {K: set() for K in Ks}
    grp = {K: dict(hr=0.0, lr=0.0, hn=0, ln=0) for K in Ks}
    high, low = set(map(int, groups_high)), set(map(int, groups_low))
    cred_sum = 0.0
    for u, cand in zip(users, cands):
        cand = np.asarray(cand, np.int64)
        scores = itf[cand] @ uf[int(u)]
        ranked = cand[np.argsort(-scores, kind="stable")]
        cred_sum += float(cred[int(u)])
        for K in Ks:
            topk = ranked[:K]
            p, r, nd = metrics_at_k(ranked, {int(cand[0])}, K)
            sums[K]["p"] += p
            sums[K]["r"] += r
            sums[K]["n"] += nd
            rec[K].update(map(int, topk.tolist()))
            pops = item_pop[topk]
            sums[K]["lp"] += float(np.log(pops + 1.0).mean())
            sums[K]["si"] += float((-np.log2((pops + 1.0) / (total_train + num_items))).mean())
            if int(u) in high:
                grp[K]["hr"] += r
                grp[K]["hn"] += 1
            if int(u) in low:
                grp[K]["lr"] += r
                grp[K]["ln"] += 1
    n = len(users)
    out = {}
    for K in Ks:
        out[K] = dict(precision=sums[K]["p"] / n, recall=sums[K]["r"] / n, ndcg=sums[K]["n"] / n,
                      item_coverage=len(rec[K]) / num_items,
                      avg_log_popularity=sums[K]["lp"] / n,
                      avg_self_information=sums[K]["si"] / n, cred_utility=cred_sum / n,
                      high_cred_recall=grp[K]["hr"] / max(grp[K]["hn"], 1),
                      low_cred_recall=grp[K]["lr"] / max(grp[K]["ln"], 1),
                      high_users=grp[K]["hn"], low_users=grp[K]["ln"])
    return out


def make_cred_groups(users, cred, pct):
    """Version-2/lighgcn_cu_pop.py:405-422 (argsort ascending; top / bottom k)."""
    users = np.asarray(users, np.int64)
    if users.size == 0:
        return np.array([], np.int64), np.array([], np.int64)
    k = max(int(round(users.size * pct)), 1)
    order = np.argsort(np.asarray(cred)[users])
    return users[order[-k:]], users[order[:k]]


def sampled_candidates_reference_style(rng, users, tr_ptr, tr_idx, te_ptr, te_idx, num_items,
                                       n_neg=99):
    """The candidate draws of the reference's loop (Version-2:575-589), literal:
    per user in order, pos = gt[rng.integers(0, len(gt))], then negatives by
    rejection on gt_set and user_has_item. Advances `rng` as the reference
    does; returns [n_users, 1 + n_neg] int64."""
    cands = []
    for u in users:
        gt = te_idx[te_ptr[u]:te_ptr[u + 1]]
        gt_set = set(map(int, gt.tolist()))
        pos = int(gt[rng.integers(0, len(gt))])
        negs = []
        while len(negs) < n_neg:
            j = int(rng.integers(0, num_items))
            if j in gt_set:
                continue
            if user_has_item(tr_ptr, tr_idx, int(u), j):
                continue
            negs.append(j)
        cands.append([pos] + negs)
    return np.asarray(cands, np.int64).reshape(len(users), 1 + n_neg)


def evaluate_sampled_reference_style(tr_ptr, tr_idx, te_ptr, te_idx, uf, itf, num_items, item_pop,
                                     total_train, cred, Ks=(10, 20), n_neg=99, pct=0.2, seed=1041,
                                     users=None, rng=None):
    """The whole reference loop (Version-2:536-650) including its numpy
    sampling stream (default_rng(seed); pos via integers(0, len(gt)); negatives
    by rejection on gt_set and user_has_item). `users` restricts the loop to a
    subset (the CPU-baseline sample); `rng` (optional) is the Generator to draw
    from, left in its end state; returns (results, candidates)."""
    rng = np.random.default_rng(seed) if rng is None else rng
    if users is None:
        users = np.where(np.diff(te_ptr) > 0)[0].astype(np.int64)
    cands = []
    for u in users:
        gt = te_idx[te_ptr[u]:te_ptr[u + 1]]
        gt_set = set(map(int, gt.tolist()))
        pos = int(gt[rng.integers(0, len(gt))])
        negs = []
        while len(negs) < n_neg:
            j = int(rng.integers(0, num_items))
            if j in gt_set or user_has_item(tr_ptr, tr_idx, int(u), j):
                continue
            negs.append(j)
        cands.append([pos] + negs)
    high, low = make_cred_groups(users, cred, pct)
    res = evaluate_sampled_given(users, np.asarray(cands, np.int64).reshape(len(users), 1 + n_neg),
                                 uf, itf, item_pop, total_train, num_items, cred, high, low, Ks)
    return res, cands


def evaluate_given_topk(users, topk, te_ptr, te_idx, item_pop, total_train, num_items, cred,
                        groups_high, groups_low, Ks=(10, 20), mode="full"):
    """The reference's metric loop (Version-2:690-752 full / :600-650 sampled)
    on FIXED ranked lists topk[b] (>= max(Ks) items, -1 padded); gt = the
    user's test row (full ranking)."""
    item_pop = np.asarray(item_pop, np.float64)
    sums = {K: dict(p=0.0, r=0.0, n=0.0, lp=0.0, si=0.0) for K in Ks}
    rec = {K: set() for K in Ks}
    grp = {K: dict(hr=0.0, lr=0.0, hn=0, ln=0) for K in Ks}
    high, low = set(map(int, groups_high)), set(map(int, groups_low))
    cred_sum = 0.0
    for u, ranked in zip(users, topk):
        gt = set(map(int, te_idx[te_ptr[u]:te_ptr[u + 1]].tolist()))
        ranked = np.asarray([x for x in ranked if x >= 0], np.int64)
        cred_sum += float(cred[int(u)])
        for K in Ks:
            top = ranked[:K]
            p, r, nd = metrics_at_k(ranked, gt, K)
            sums[K]["p"] += p
            sums[K]["r"] += r
            sums[K]["n"] += nd
            rec[K].update(map(int, top.tolist()))
            if top.size:
                pops = item_pop[top]
                sums[K]["lp"] += float(np.log(pops + 1.0).mean())
                sums[K]["si"] += float((-np.log2((pops + 1.0) / (total_train + num_items))).mean())
            if int(u) in high:
                grp[K]["hr"] += r
                grp[K]["hn"] += 1
            if int(u) in low:
                grp[K]["lr"] += r
                grp[K]["ln"] += 1
    n = len(users)
    return {K: dict(precision=sums[K]["p"] / n, recall=sums[K]["r"] / n, ndcg=sums[K]["n"] / n,
                    item_coverage=len(rec[K]) / num_items,
                    avg_log_popularity=sums[K]["lp"] / n,
                    avg_self_information=sums[K]["si"] / n, cred_utility=cred_sum / n,
                    high_cred_recall=grp[K]["hr"] / max(grp[K]["hn"], 1),
                    low_cred_recall=grp[K]["lr"] / max(grp[K]["ln"], 1),
                    high_users=grp[K]["hn"], low_users=grp[K]["ln"]) for K in Ks}


def full_ranking_reference_style(users, tr_ptr, tr_idx, uf, itf, k):
    """The reference's per-user full ranking (Version-2:690-706): fp32 scores
    over every item, train items at -1e9, argsort descending (stable here:
    ties by item id), top-k. Returns [n, k] int64."""
    itf = np.asarray(itf, np.float32)
    out = np.empty((len(users), k), np.int64)
    for b, u in enumerate(users):
        scores = (np.asarray(uf[int(u)], np.float32)[None, :] * itf).sum(axis=1)
        tr = tr_idx[tr_ptr[u]:tr_ptr[u + 1]]
        if tr.size:
            scores[tr] = np.float32(-1e9)
        out[b] = np.argsort(-scores, kind="stable")[:k]
    return out


# ---------------------------------------------------------------------------
# Credibility GNN edge weighting + aggregation (main.py:677-691)
# ---------------------------------------------------------------------------
def ewa_raw(edge_attr, col_verified=0, col_align=1, beta=1.0, gamma=1.0):
    """main.py:677-681: clamp(beta*clamp(verified,0,1) + gamma*align, min=0),
    evaluated in fp32 as torch does."""
    a = np.asarray(edge_attr, np.float32)
    v = np.clip(a[:, col_verified], np.float32(0), np.float32(1))
    w = np.float32(beta) * v + np.float32(gamma) * a[:, col_align]
    return np.maximum(w, np.float32(0)).astype(np.float32)


def normalize_per_dst(w, dst, num_dst, eps=1e-12):
    """main.py:683-685 in float64: w / (sum of w over dst + eps)[dst]."""
    w = np.asarray(w, np.float64)
    den = np.zeros(num_dst, np.float64)
    np.add.at(den, np.asarray(dst), w)
    return w / (den + eps)[np.asarray(dst)]


def aggregate(src_x, edge_index, w_tilde, num_dst):
    """main.py:687-691 in float64: scatter_add(w_tilde * src_x[src], dst)."""
    x = np.asarray(src_x, np.float64)
    src, dst = np.asarray(edge_index[0]), np.asarray(edge_index[1])
    out = np.zeros((num_dst, x.shape[1]), np.float64)
    np.add.at(out, dst, np.asarray(w_tilde, np.float64)[:, None] * x[src])
    return out
