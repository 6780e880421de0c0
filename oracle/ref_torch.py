"""ORACLE (test infrastructure only): fp32 torch restatement of the reference
hot path, built from the same torch calls the reference makes, so that its
CPU timing is a faithful "reference CPU path" (bench.py cpu_baseline) and its
autograd gives an independent gradient reference.

  operators   sparse_coo_tensor(...).coalesce()   Version-2/lighgcn_cu_pop.py:441-450
  propagate   torch.sparse.mm per layer + stack().mean(0)   :482-489
  loss        -log(sigmoid(s+ - s-) + 1e-12).mean() + reg * ego L2   :496-507
  optimizer   torch.optim.Adam(lr)                           :793, :861-863
"""
from __future__ import annotations

import numpy as np
import torch

from . import ref_numpy


def coo(rows, cols, vals, shape, device="cpu"):
    idx = torch.tensor(np.vstack([rows, cols]), dtype=torch.long, device=device)
    val = torch.tensor(np.asarray(vals, np.float32), dtype=torch.float32, device=device)
    return torch.sparse_coo_tensor(idx, val, size=shape).coalesce()


def gs_operators(edges, U, I, cred_u=None, method_a=False, device="cpu"):
    """(M_ui [U,I], M_iu [I,U]) — Version-2/lighgcn_cu_pop.py:429-452."""
    u, i, w_ui, w_iu = ref_numpy.gs_values(edges, U, I, cred_u, method_a)
    return coo(u, i, w_ui, (U, I), device), coo(i, u, w_iu, (I, U), device)


def j_operators(edges, U, I, cred_u=None, device="cpu"):
    """(M_ui [I,U] item<-user, M_iu [U,I] user<-item) — lightgcn_cu.py:368-399."""
    u, i, w_ui, w_iu, _ = ref_numpy.j_values(edges, U, I, cred_u)
    return coo(i, u, w_ui, (I, U), device), coo(u, i, w_iu, (U, I), device)


def sym_operator(edges, U, I, device="cpu"):
    """A_hat [N,N] — lightgcn.py:352-372 (torch calls as in the reference)."""
    u = edges[0].astype(np.int64)
    it = edges[1].astype(np.int64) + U
    row, col = np.concatenate([u, it]), np.concatenate([it, u])
    N = U + I
    adj = coo(row, col, np.ones(row.size, np.float32), (N, N), device)
    deg = torch.sparse.sum(adj, dim=1).to_dense()
    dinv = torch.pow(deg, -0.5)
    dinv[torch.isinf(dinv)] = 0.0
    r, c = adj.indices()
    v = adj.values() * dinv[r] * dinv[c]
    return torch.sparse_coo_tensor(adj.indices(), v, size=adj.size()).coalesce()


def propagate_gs(M_ui, M_iu, u0, i0, K):
    u_list, i_list = [u0], [i0]
    u, i = u0, i0
    for _ in range(K):
        i = torch.sparse.mm(M_iu, u)
        u = torch.sparse.mm(M_ui, i)
        u_list.append(u)
        i_list.append(i)
    return torch.stack(u_list, 0).mean(0), torch.stack(i_list, 0).mean(0)


def propagate_j(M_item_from_user, M_user_from_item, u0, i0, K):
    us, is_ = [u0], [i0]
    for _ in range(K):
        e_i = torch.sparse.mm(M_item_from_user, us[-1])
        e_u = torch.sparse.mm(M_user_from_item, is_[-1])
        us.append(e_u)
        is_.append(e_i)
    return torch.stack(us, 0).mean(0), torch.stack(is_, 0).mean(0)


def propagate_sym(A, x0, K):
    xs, x = [x0], x0
    for _ in range(K):
        x = torch.sparse.mm(A, x)
        xs.append(x)
    return torch.stack(xs, 0).mean(0)


def bpr(uf, itf, ue, ie, users, pos, neg, reg, pop=None, lambda_fair=0.0):
    u, p, n = uf[users], itf[pos], itf[neg]
    ps, ns = (u * p).sum(1), (u * n).sum(1)
    loss = -torch.log(torch.sigmoid(ps - ns) + 1e-12).mean()
    r = (ue[users].norm(2, dim=1).pow(2) + ie[pos].norm(2, dim=1).pow(2)
         + ie[neg].norm(2, dim=1).pow(2)).mean()
    loss = loss + reg * r
    if pop is not None:
        loss = loss + lambda_fair * (pop[pos] * ps).mean()
    return loss


class GSModel(torch.nn.Module):
    """Version-2 LightGCN restated (user_emb / item_emb, GS order)."""

    def __init__(self, U, I, d, K, M_ui, M_iu, u0=None, i0=None):
        super().__init__()
        self.K, self.M_ui, self.M_iu = K, M_ui, M_iu
        self.user_emb = torch.nn.Embedding(U, d)
        self.item_emb = torch.nn.Embedding(I, d)
        with torch.no_grad():
            if u0 is not None:
                self.user_emb.weight.copy_(torch.as_tensor(u0))
                self.item_emb.weight.copy_(torch.as_tensor(i0))
            else:
                torch.nn.init.xavier_uniform_(self.user_emb.weight)
                torch.nn.init.xavier_uniform_(self.item_emb.weight)

    def finals(self):
        return propagate_gs(self.M_ui, self.M_iu, self.user_emb.weight,
                            self.item_emb.weight, self.K)

    def loss(self, users, pos, neg, reg):
        uf, itf = self.finals()
        return bpr(uf, itf, self.user_emb.weight, self.item_emb.weight, users, pos, neg, reg)


class JModel(GSModel):
    """lightgcn_cu.py CredLightGCN restated: Jacobi layers (:420-448), the BPR
    loss + lambda_fair * L_fair (pop[pos] * s+) + reg * ego L2 (:632-648)."""

    def __init__(self, U, I, d, K, M_item_from_user, M_user_from_item, pop, lambda_fair):
        super().__init__(U, I, d, K, M_user_from_item, M_item_from_user)
        self.pop, self.lambda_fair = pop, lambda_fair

    def finals(self):
        return propagate_j(self.M_iu, self.M_ui, self.user_emb.weight, self.item_emb.weight,
                           self.K)

    def loss(self, users, pos, neg, reg):
        uf, itf = self.finals()
        return bpr(uf, itf, self.user_emb.weight, self.item_emb.weight, users, pos, neg, reg,
                   self.pop, self.lambda_fair)


class SymModel(torch.nn.Module):
    """lightgcn.py LightGCN restated: one emb [N, d] (:306-316), x_{k+1} = A_hat
    x_k (:318-325), the BPR loss with the ego rows at offset U (:333-349)."""

    def __init__(self, U, I, d, K, A):
        super().__init__()
        self.U, self.K, self.A = U, K, A
        self.emb = torch.nn.Embedding(U + I, d)
        torch.nn.init.xavier_uniform_(self.emb.weight)

    def finals(self):
        x = propagate_sym(self.A, self.emb.weight, self.K)
        return x[: self.U], x[self.U:]

    def loss(self, users, pos, neg, reg):
        uf, itf = self.finals()
        W = self.emb.weight
        return bpr(uf, itf, W[: self.U], W[self.U:], users, pos, neg, reg)


def reference_model(variant: str, edges, U, I, d, K, cred=None, lambda_fair=0.05):
    """(model, uses popularity-mix negatives) of one reference family, with the
    family's own operator builder: "v2_pop" / "cu_message" (Version-2 /
    version_1 GS), "method_a", "cu_fair" (lightgcn_cu.py), "plain" (lightgcn.py)."""
    if variant in ("v2_pop", "cu_message", "method_a"):
        M_ui, M_iu = gs_operators(edges, U, I, cred, method_a=variant == "method_a")
        return GSModel(U, I, d, K, M_ui, M_iu), variant == "v2_pop"
    if variant == "cu_fair":
        a, b = j_operators(edges, U, I, cred)
        deg_i = np.bincount(edges[1].astype(np.int64), minlength=I).astype(np.float32)
        pop = torch.as_tensor(deg_i / max(float(deg_i.max()), 1.0))
        return JModel(U, I, d, K, a, b, pop, lambda_fair), False
    if variant == "plain":
        return SymModel(U, I, d, K, sym_operator(edges, U, I)), False
    raise ValueError(f"unknown variant {variant!r}")


def train_step(model: GSModel, opt: torch.optim.Optimizer, users, pos, neg, reg):
    """One reference training step (Version-2/lighgcn_cu_pop.py:858-865)."""
    loss = model.loss(users, pos, neg, reg)
    opt.zero_grad()
    loss.backward()
    opt.step()
    return float(loss.item())


class CredModelRef(torch.nn.Module):
    """fp32 torch restatement of main.py:659-707 (CredModel) with the
    reference's own expressions (index_add_ scatter, per-dst normalisation):
    the CPU model the device CredModel is checked against."""

    def __init__(self, user_in_dim, item_in_dim, hidden_dim, col_verified=0, col_align=1,
                 beta=1.0, gamma=1.0):
        super().__init__()
        nn = torch.nn
        self.user_proj = nn.Linear(user_in_dim, hidden_dim)
        self.item_proj = nn.Linear(item_in_dim, hidden_dim)
        self.item_upd = nn.Linear(hidden_dim * 2, hidden_dim)
        self.user_upd = nn.Linear(hidden_dim * 2, hidden_dim)
        self.out = nn.Linear(hidden_dim, 1)
        self.cv, self.ca, self.beta, self.gamma = col_verified, col_align, beta, gamma

    @staticmethod
    def _scatter_add(src, index, dim_size):
        out = torch.zeros((dim_size,) + src.shape[1:], dtype=src.dtype)
        out.index_add_(0, index, src)
        return out

    def ewa_raw(self, ea):
        w = self.beta * ea[:, self.cv].clamp(0, 1) + self.gamma * ea[:, self.ca]
        return w.clamp(min=0.0)

    def normalize_per_dst(self, w, dst, num_dst):
        denom = self._scatter_add(w.unsqueeze(-1), dst, num_dst).squeeze(-1) + 1e-12
        return w / denom[dst]

    def aggregate(self, src_x, edge_index, w_tilde, num_dst):
        msg = w_tilde.unsqueeze(-1) * src_x[edge_index[0]]
        return self._scatter_add(msg, edge_index[1], num_dst)

    def forward_subgraph(self, x_u, x_i, e_u2i, ea_u2i, e_i2u, ea_i2u):
        F = torch.nn.functional
        h_u0, h_i0 = self.user_proj(x_u), self.item_proj(x_i)
        w1t = self.normalize_per_dst(self.ewa_raw(ea_u2i), e_u2i[1], h_i0.size(0))
        h_i1 = F.relu(self.item_upd(torch.cat([h_i0, self.aggregate(h_u0, e_u2i, w1t,
                                                                  h_i0.size(0))], -1)))
        w2t = self.normalize_per_dst(self.ewa_raw(ea_i2u), e_i2u[1], h_u0.size(0))
        h_u2 = F.relu(self.user_upd(torch.cat([h_u0, self.aggregate(h_i1, e_i2u, w2t,
                                                                  h_u0.size(0))], -1)))
        return torch.sigmoid(self.out(h_u2)).squeeze(-1), h_u2, h_i1, w1t
