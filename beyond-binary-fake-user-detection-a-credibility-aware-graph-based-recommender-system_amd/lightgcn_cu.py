"""Drop-in for the model layer of lightgcn_cu.py (thesis Eq 3.22-3.28).

  build_cred_weighted_mats(train_edges, num_users, num_items, cred_u, device)
      -> (M_ui [I x U] item<-user with credibility, M_iu [U x I], deg_i)
      NOTE the reference's names are swapped relative to Version-2
      (lightgcn_cu.py:368-399); this module keeps them exactly.
  CredLightGCN(num_users, num_items, emb_dim, num_layers, M_ui, M_iu)
      .propagate_all_layers() -> ([e_u^0..e_u^K], [e_i^0..e_i^K])  Jacobi order
      .final_embeddings() -> layer means (fused kernel path)
      .score(users, items, e_u, e_i); .l2_reg(users, pos, neg)
  bpr_fair_loss(...) — the fused form of :635-648 (BPR + lambda_fair * L_fair
      + lambda_reg * L_reg) with L_fair = mean(pop[pos] * pos_score).
"""
from __future__ import annotations

import numpy as np
import torch

from . import bpr as _bpr
# the reference module's host CSR helpers / samplers, bit-exact (numpy stream
# included) and O(log I) per popularity draw: bbgr.host_sampler
from .host_sampler import (edges_to_user_csr, sample_neg_item, sample_pos_item,
                           user_has_item)  # noqa: F401
from ._lib import OP_J
from .operators import (ITEM_FROM_USER, USER_FROM_ITEM, BipartiteOperator, build_pair,
                        input_order_vector, resolve_pair)
from .propagate import ORDER_J, OperatorPair, propagate as _propagate


def build_cred_weighted_mats(train_edges, num_users: int, num_items: int,
                             cred_u: np.ndarray, device: str):
    """Eq 3.23: M_ui[i,u] = c_u / sqrt(deg_u deg_i); Eq 3.24: M_iu[u,i] = 1/sqrt(..)."""
    graph, sc, pair = build_pair(train_edges, num_users, num_items, OP_J, cred_u, device)
    M_ui = BipartiteOperator(pair, ITEM_FROM_USER, graph, OP_J)   # [I, U]
    M_iu = BipartiteOperator(pair, USER_FROM_ITEM, graph, OP_J)   # [U, I]
    deg_i = input_order_vector(graph, sc.deg_i, "item").detach().cpu().numpy().astype(np.float32)
    return M_ui, M_iu, deg_i


class CredLightGCN(torch.nn.Module):
    def __init__(self, num_users, num_items, emb_dim, num_layers, M_ui, M_iu):
        super().__init__()
        self.num_users = num_users
        self.num_items = num_items
        self.num_layers = num_layers
        self.M_ui = M_ui.coalesce()
        self.M_iu = M_iu.coalesce()
        self._pair: OperatorPair | None = None

        self.user_emb = torch.nn.Embedding(num_users, emb_dim)
        self.item_emb = torch.nn.Embedding(num_items, emb_dim)
        torch.nn.init.xavier_uniform_(self.user_emb.weight)
        torch.nn.init.xavier_uniform_(self.item_emb.weight)

    def _operator_pair(self) -> OperatorPair:
        if self._pair is None:
            # here M_ui is item<-user [I,U] and M_iu is user<-item [U,I]
            self._pair = resolve_pair(self.M_ui, self.M_iu, self.num_users, self.num_items,
                                      self.user_emb.weight.device)
        return self._pair

    def propagate_all_layers(self):
        """Per-layer tables (unfused; one SpMM per side per layer)."""
        pair = self._operator_pair()
        e_u, e_i = self.user_emb.weight, self.item_emb.weight
        us, is_ = [e_u], [e_i]
        for _ in range(self.num_layers):
            # Eq 3.23 item <- user (cred); Eq 3.24 user <- item uses is_[-1]
            new_i, new_u = _propagate_one(pair, us[-1], is_[-1])
            us.append(new_u)
            is_.append(new_i)
        return us, is_

    def final_embeddings(self):
        return _propagate(self._operator_pair(), self.user_emb.weight, self.item_emb.weight,
                          self.num_layers, ORDER_J)

    def score(self, users: torch.Tensor, items: torch.Tensor, e_u: torch.Tensor,
              e_i: torch.Tensor):
        return (e_u[users] * e_i[items]).sum(dim=1)

    def l2_reg(self, users, pos_items, neg_items):
        eu = self.user_emb.weight[users]
        ep = self.item_emb.weight[pos_items]
        en = self.item_emb.weight[neg_items]
        return (eu.norm(2, dim=1).pow(2) + ep.norm(2, dim=1).pow(2)
                + en.norm(2, dim=1).pow(2)).mean()

    def bpr_fair_loss(self, users, pos_items, neg_items, e_u, e_i, pop: torch.Tensor,
                      lambda_fair: float, lambda_reg: float):
        """loss_bpr + lambda_fair * mean(pop[pos]*pos_score) + lambda_reg * l2_reg,
        one fused kernel (lightgcn_cu.py:635-648)."""
        return _bpr.bpr_loss(users, pos_items, neg_items, e_u, e_i, self.user_emb.weight,
                             self.item_emb.weight, lambda_reg,
                             pop.to(device=e_u.device, dtype=torch.float32).contiguous(),
                             lambda_fair)


def _propagate_one(pair: OperatorPair, u: torch.Tensor, i: torch.Tensor):
    """One Jacobi layer (i' = M_ui u, u' = M_iu i) as a differentiable op:
    the registered operator bbgr::jacobi_layer (ops.py)."""
    from . import ops
    return ops.jacobi_layer(u, i, ops.pair_key(pair))


__all__ = ["build_cred_weighted_mats", "CredLightGCN", "evaluate_sampled"]


def evaluate_sampled(model, train_csr, test_csr, num_items: int, device: str, **cfg):
    """lightgcn_cu.py:487-547 (same arguments; precision / recall / ndcg per K):
    bbgr.evaluation.evaluate_sampled, candidates drawn on the device."""
    from .evaluation import evaluate_sampled_reference
    return evaluate_sampled_reference(model, train_csr, test_csr, num_items, device, **cfg)
