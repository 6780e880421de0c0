"""Drop-in for the model layer of Version-2/lighgcn_cu_pop.py.

Same names, signatures, attributes and state_dict keys as the reference:

  build_message_passing_mats(train_edges_2xE, num_users, num_items, cred_u, device)
      -> (M_ui [U x I], M_iu [I x U])          Version-2/lighgcn_cu_pop.py:429-452
  LightGCN(num_users, num_items, emb_dim, num_layers, M_ui, M_iu)   :458-508
      .user_emb / .item_emb (nn.Embedding, xavier_uniform_), .M_ui, .M_iu,
      .propagate() -> (u_final, i_final)   Gauss-Seidel order (:472-490)
      .get_user_item_emb()
      .bpr_loss(users, pos_items, neg_items, user_emb, item_emb, reg_weight)
  state_dict keys: user_emb.weight, item_emb.weight (the operators are plain
  attributes, not buffers, as in the reference).

The operators are built ON the device from the int32 [2, E] edge array; no
numpy weight math, no COO coalesce. The graph inside is numbered by
descending degree (operators.DROPIN_VERTEX_ORDER) while the embedding tables,
the final tables and the gradients stay in the caller's ids. Torch sparse COO operators are also
accepted by LightGCN (converted once to explicit-value CSRs).
"""
from __future__ import annotations

import torch

from . import bpr as _bpr
# the reference module's host CSR helpers / samplers, bit-exact (numpy stream
# included) and O(log I) per popularity draw: bbgr.host_sampler
from .host_sampler import (edges_to_user_csr, sample_neg_item_popmix, sample_pos_item,
                           user_has_item)  # noqa: F401
from . import lazy as _lazy
from ._lib import OP_GS
from .operators import (ITEM_FROM_USER, USER_FROM_ITEM, BipartiteOperator, build_pair,
                        resolve_pair)
from .propagate import ORDER_GS, OperatorPair, propagate as _propagate
from .propagate import propagate_rows as _propagate_rows


def _build(train_edges_2xE, num_users, num_items, cred_u, device, kind):
    graph, sc, pair = build_pair(train_edges_2xE, num_users, num_items, kind, cred_u, device)
    M_ui = BipartiteOperator(pair, USER_FROM_ITEM, graph, kind)
    M_iu = BipartiteOperator(pair, ITEM_FROM_USER, graph, kind)
    return M_ui, M_iu


def build_message_passing_mats(train_edges_2xE, num_users: int, num_items: int,
                               cred_u: torch.Tensor, device: str):
    """M_ui[u,i] = w_ui, M_iu[i,u] = c_u * w_ui,
    w_ui = (1/sqrt(max(deg_u,1))) * (1/sqrt(max(deg_i,1)))  (Version-2:429-452)."""
    return _build(train_edges_2xE, num_users, num_items, cred_u, device, OP_GS)


class LightGCN(torch.nn.Module):
    # propagate() returns deferred tables (bbgr.lazy): bpr_loss over one call's
    # pair computes the batch rows only; any other use computes them whole
    lazy_finals = True

    def __init__(self, num_users, num_items, emb_dim, num_layers, M_ui, M_iu):
        super().__init__()
        self.num_users = num_users
        self.num_items = num_items
        self.num_layers = num_layers
        self.M_ui = M_ui
        self.M_iu = M_iu
        self._pair: OperatorPair | None = None

        self.user_emb = torch.nn.Embedding(num_users, emb_dim)
        self.item_emb = torch.nn.Embedding(num_items, emb_dim)
        torch.nn.init.xavier_uniform_(self.user_emb.weight)
        torch.nn.init.xavier_uniform_(self.item_emb.weight)

    def _operator_pair(self) -> OperatorPair:
        if self._pair is None:
            self._pair = resolve_pair(self.M_iu, self.M_ui, self.num_users, self.num_items,
                                      self.user_emb.weight.device)
        return self._pair

    def propagate(self):
        pair, K = self._operator_pair(), self.num_layers
        u0, i0 = self.user_emb.weight, self.item_emb.weight
        if self.lazy_finals and _lazy.supported(u0, i0):
            from .ops import pair_key
            return _lazy.deferred_pair(
                lambda: _propagate(pair, u0, i0, K, ORDER_GS),
                lambda users, items: _propagate_rows(pair, u0, i0, K, ORDER_GS, users, items),
                u0, i0, step=(pair_key(pair), K,
                              (pair.io.user_map64, pair.io.item_map64) if pair.io else None))
        return _propagate(pair, u0, i0, K, ORDER_GS)

    def get_user_item_emb(self):
        return self.propagate()

    def bpr_loss(self, users, pos_items, neg_items, user_emb, item_emb, reg_weight: float):
        # bbgr.optim.FusedAdam(fuse_backward=True) on both tables: the backward
        # of this loss runs the optimizer step (lazy.fused_bpr_step)
        fused = _lazy.fused_bpr_step(user_emb, item_emb, users, pos_items, neg_items,
                                     reg_weight)
        if fused is not None:
            return fused
        user_emb, item_emb, users, pos_items, neg_items = _lazy.batch_finals(
            user_emb, item_emb, users, pos_items, neg_items)
        return _bpr.bpr_loss(users, pos_items, neg_items, user_emb, item_emb,
                             self.user_emb.weight, self.item_emb.weight, reg_weight)


def evaluate_sampled(model, train_csr, test_csr, num_items: int, device: str, item_pop,
                     total_train_interactions: int, cred_np, **cfg):
    """Version-2/lighgcn_cu_pop.py:536-650 (same arguments, the same result
    dictionary per K; cfg.Ks / sampled_negatives / cred_group_pct / seed as
    keyword arguments): one device launch for all users
    (bbgr.evaluation.evaluate_sampled; candidates drawn by Philox)."""
    from .evaluation import evaluate_sampled_reference
    return evaluate_sampled_reference(model, train_csr, test_csr, num_items, device, item_pop,
                                      total_train_interactions, cred_np, **cfg)


def evaluate_full_ranking(model, train_csr, test_csr, num_items: int, device: str, item_pop,
                          total_train_interactions: int, cred_np, **cfg):
    """Version-2/lighgcn_cu_pop.py:653-752 (same arguments and result
    dictionary): fp32 MFMA scores with the train items masked and a running
    top-K (bbgr.evaluation.evaluate_full)."""
    from .evaluation import evaluate_full_ranking_reference
    return evaluate_full_ranking_reference(model, train_csr, test_csr, num_items, device,
                                           item_pop, total_train_interactions, cred_np, **cfg)
