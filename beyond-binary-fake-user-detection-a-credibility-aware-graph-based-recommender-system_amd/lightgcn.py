"""Drop-in for the model layer of lightgcn.py / lightgcn-1.py (plain LightGCN).

  build_norm_adj(train_edges, num_users, num_items, device) -> A_hat [N x N]
      D^-1/2 A D^-1/2 of the symmetric bipartite adjacency, isolated nodes 0
      (lightgcn.py:352-372). Held as its two off-diagonal blocks.
  LightGCN(num_users, num_items, emb_dim, num_layers, norm_adj)   :306-349
      .emb (nn.Embedding(N, d)), .propagate() -> x_final [N, d],
      .get_user_item_emb() -> (x_final[:U], x_final[U:]),
      .bpr_loss(...) with ego rows emb.weight[users], emb.weight[U + items].
  state_dict key: emb.weight.

x_k = A_hat x_{k-1} on the block form is the Jacobi order over the two
bipartite blocks; user/item halves of the [N, d] tables are row-offset views.
A torch sparse COO norm_adj of any N x N pattern is also accepted.
"""
from __future__ import annotations

import torch

from . import bpr as _bpr
# the reference module's host CSR helpers / samplers, bit-exact (numpy stream
# included) and O(log I) per popularity draw: bbgr.host_sampler
from .host_sampler import (edges_to_user_csr, sample_neg_item, sample_pos_item,
                           user_has_item)  # noqa: F401
from ._lib import OP_SYM
from .operators import NormAdjOperator, build_pair, square_from_torch_sparse
from .propagate import (ORDER_J, OperatorPair, _SquareFn, backward as _bwd,
                        forward as _fwd)


def build_norm_adj(train_edges, num_users: int, num_items: int, device):
    graph, sc, pair = build_pair(train_edges, num_users, num_items, OP_SYM, None, device)
    return NormAdjOperator(pair, graph)


class LightGCN(torch.nn.Module):
    def __init__(self, num_users, num_items, emb_dim, num_layers, norm_adj):
        super().__init__()
        self.num_users = num_users
        self.num_items = num_items
        self.num_nodes = num_users + num_items
        self.num_layers = num_layers
        self.norm_adj = norm_adj
        self._square = None

        self.emb = torch.nn.Embedding(self.num_nodes, emb_dim)
        torch.nn.init.xavier_uniform_(self.emb.weight)

    def propagate(self):
        if isinstance(self.norm_adj, NormAdjOperator):
            from . import ops
            return ops.propagate_sym(self.emb.weight, ops.pair_key(self.norm_adj.pair),
                                     int(self.num_layers))
        if self._square is None:
            self._square = square_from_torch_sparse(self.norm_adj, self.emb.weight.device)
        return _SquareFn.apply(self.emb.weight, self._square, self.num_layers)

    def get_user_item_emb(self):
        x_final = self.propagate()
        return x_final[: self.num_users], x_final[self.num_users:]

    def bpr_loss(self, users, pos_items, neg_items, user_emb, item_emb, reg_weight: float):
        W = self.emb.weight
        return _bpr.bpr_loss(users, pos_items, neg_items, user_emb, item_emb,
                             W[: self.num_users], W[self.num_users:], reg_weight)


def evaluate_sampled(model, train_csr, test_csr, num_items: int, device: str, **cfg):
    """lightgcn.py:397-457 (same arguments; precision / recall / ndcg per K):
    bbgr.evaluation.evaluate_sampled, candidates drawn on the device."""
    from .evaluation import evaluate_sampled_reference
    return evaluate_sampled_reference(model, train_csr, test_csr, num_items, device, **cfg)


def evaluate_full_ranking(model, train_csr, test_csr, num_items: int, device: str, **cfg):
    """lightgcn.py:459-520 (same arguments; precision / recall / ndcg per K):
    bbgr.evaluation.evaluate_full."""
    from .evaluation import evaluate_full_ranking_reference
    return evaluate_full_ranking_reference(model, train_csr, test_csr, num_items, device, **cfg)
