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
from ._lib import OP_SYM
from .graph import BipartiteGraph
from .operators import NormAdjOperator, square_from_torch_sparse
from .propagate import (ORDER_J, OperatorPair, _SquareFn, backward as _bwd,
                        forward as _fwd)


def build_norm_adj(train_edges, num_users: int, num_items: int, device):
    graph = BipartiteGraph(train_edges, num_users, num_items, device)
    sc = graph.scales(OP_SYM, None)
    return NormAdjOperator(OperatorPair.factored(graph, sc), graph)


class _SymPropagateFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x0, pair, K):
        U = pair.num_users
        x0 = x0.contiguous()
        out = torch.empty_like(x0)
        _fwd(pair, x0[:U], x0[U:], K, ORDER_J, out_u=out[:U], out_i=out[U:])
        ctx.pair, ctx.K = pair, K
        return out

    @staticmethod
    def backward(ctx, g):
        pair, U = ctx.pair, ctx.pair.num_users
        g = g.contiguous()
        gx = torch.empty_like(g)
        _bwd(pair, g[:U], g[U:], ctx.K, ORDER_J, out_u=gx[:U], out_i=gx[U:])
        return gx, None, None


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
            return _SymPropagateFn.apply(self.emb.weight, self.norm_adj.pair, self.num_layers)
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
