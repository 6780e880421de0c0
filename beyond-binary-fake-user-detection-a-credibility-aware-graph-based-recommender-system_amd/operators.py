"""Operator objects returned by the build_* functions.

The reference returns coalesced torch sparse COO tensors; this package returns
``BipartiteOperator`` handles onto one shared device graph (two CSRs + scale
vectors, see graph.py). The model classes accept either: a handle pair is used
directly, a torch sparse COO pair is converted once into explicit-value CSRs
(``OperatorPair.generic``), so code that hands in its own sparse tensors keeps
working.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _lib
from .graph import BipartiteGraph, Csr
from .propagate import OperatorPair, Product, SquareOperator, spmm

ITEM_FROM_USER = "item<-user"   # shape [I, U]
USER_FROM_ITEM = "user<-item"   # shape [U, I]


class BipartiteOperator:
    """One direction of a factored operator pair: diag(row) A diag(col)."""

    def __init__(self, pair: OperatorPair, role: str, graph: BipartiteGraph | None = None,
                 kind: int | None = None):
        self.pair, self.role, self.graph, self.kind = pair, role, graph, kind
        U, I = pair.num_users, pair.num_items
        self.shape = torch.Size((I, U) if role == ITEM_FROM_USER else (U, I))

    # --- torch.sparse-like surface -------------------------------------------
    def size(self, dim: int | None = None):
        return self.shape if dim is None else self.shape[dim]

    def coalesce(self):
        return self

    def is_coalesced(self) -> bool:
        return True

    @property
    def device(self):
        return self._product.csr.device

    @property
    def _product(self) -> Product:
        return self.pair.fwd_item if self.role == ITEM_FROM_USER else self.pair.fwd_user

    def _nnz(self) -> int:
        return self._product.csr.nnz

    def mm(self, x: torch.Tensor) -> torch.Tensor:
        """y = M x (no autograd), like torch.sparse.mm(M, x)."""
        prod = self._product
        _lib.require_gpu(x)
        x = x.contiguous()
        y = torch.empty(self.shape[0], x.shape[1], dtype=torch.float32, device=x.device)
        # diag(out) A diag(in) x: first-layer form applies `in` per gathered row;
        # an input-order pair gathers x by input id and places y's rows by map
        io = self.pair.io
        y_map = None if io is None else (io.item_map if self.role == ITEM_FROM_USER
                                         else io.user_map)
        spmm(prod, x, True, y=y, y_scale=prod.out_scale, src_input=io is not None,
             y_map=y_map)
        return y

    __matmul__ = mm

    def to_torch_sparse(self) -> torch.Tensor:
        """Coalesced COO with the reference's values (for inspection/tests)."""
        prod = self._product
        csr = prod.csr
        rows = torch.repeat_interleave(
            torch.arange(csr.n_rows, device=csr.device),
            (csr.indptr[1:] - csr.indptr[:-1]).long())
        cols = csr.indices[: csr.nnz].long()
        if prod.vals is not None:
            vals = prod.vals[: csr.nnz]
        else:
            vals = prod.out_scale[rows] * prod.in_scale[cols]
        io = self.pair.io
        if io is not None:   # internal ids -> the caller's input ids
            rmap, cmap = ((io.item_map64, io.user_map64) if self.role == ITEM_FROM_USER
                          else (io.user_map64, io.item_map64))
            rows, cols = rmap[rows], cmap[cols]
        return torch.sparse_coo_tensor(torch.stack([rows, cols]), vals,
                                       size=self.shape).coalesce()


class NormAdjOperator:
    """lightgcn.py's N x N symmetric A_hat, held as its two bipartite blocks."""

    def __init__(self, pair: OperatorPair, graph: BipartiteGraph):
        self.pair, self.graph = pair, graph
        self.num_users, self.num_items = pair.num_users, pair.num_items
        n = self.num_users + self.num_items
        self.shape = torch.Size((n, n))

    def size(self, dim: int | None = None):
        return self.shape if dim is None else self.shape[dim]

    def coalesce(self):
        return self

    def to_torch_sparse(self) -> torch.Tensor:
        U = self.num_users
        a = BipartiteOperator(self.pair, ITEM_FROM_USER).to_torch_sparse()
        b = BipartiteOperator(self.pair, USER_FROM_ITEM).to_torch_sparse()
        ai, bi = a.indices(), b.indices()
        idx = torch.cat([torch.stack([ai[0] + U, ai[1]]), torch.stack([bi[0], bi[1] + U])], 1)
        vals = torch.cat([a.values(), b.values()])
        return torch.sparse_coo_tensor(idx, vals, size=self.shape).coalesce()


# Vertex order of the graphs the drop-in builders make: "degree" numbers users
# and items by descending degree inside the graph (hot rows cached, cold rows
# streamed) while every table the caller sees stays in its input
# order (OperatorPair.set_input_order); each row keeps its input-order column
# sequence, so results are bitwise those of an input-order build. "input":
# the graph in the caller's numbering (BBGR_DROPIN_ORDER=input, A/B runs).
DROPIN_VERTEX_ORDER = os.environ.get("BBGR_DROPIN_ORDER", "degree")


def build_pair(train_edges, num_users: int, num_items: int, kind: int, cred_u, device):
    """(graph, scales, pair) of a drop-in builder: the device graph, the
    operator family's scale vectors and the factored pair, with the caller's
    input-order credibility vector (None: no credibility)."""
    graph = BipartiteGraph(train_edges, num_users, num_items, device,
                           vertex_order=DROPIN_VERTEX_ORDER, input_col_order=True)
    cred = to_device_cred(cred_u, num_users, graph.device)
    if cred is not None and graph.user_order is not None:
        cred = cred[graph.user_order._perm64].contiguous()   # internal order
    sc = graph.scales(kind, cred)
    pair = OperatorPair.factored(graph, sc)
    if graph.user_order is not None:
        pair.set_input_order(graph.user_order, graph.item_order)
    return graph, sc, pair


def input_order_vector(graph: BipartiteGraph, v: torch.Tensor, side: str) -> torch.Tensor:
    """A per-item / per-user vector of the graph (internal order) by input id."""
    order = graph.item_order if side == "item" else graph.user_order
    return v if order is None else v[order._rank64]


def _coo_parts(M: torch.Tensor):
    if not (isinstance(M, torch.Tensor) and M.layout == torch.sparse_coo):
        raise TypeError(f"expected a bbgr operator or a torch sparse COO tensor, got {type(M)}")
    M = M.coalesce()
    return M.indices(), M.values(), M.shape


def pair_from_torch_sparse(item_from_user: torch.Tensor, user_from_item: torch.Tensor,
                           num_users: int, num_items: int, device) -> OperatorPair:
    """Explicit-value operator pair from two torch COO tensors ([I,U] and [U,I])."""
    (iu_idx, iu_val, iu_shape) = _coo_parts(item_from_user)
    (ui_idx, ui_val, ui_shape) = _coo_parts(user_from_item)
    if tuple(iu_shape) != (num_items, num_users) or tuple(ui_shape) != (num_users, num_items):
        raise ValueError(f"operator shapes {tuple(iu_shape)} / {tuple(ui_shape)} do not match "
                         f"({num_items},{num_users}) / ({num_users},{num_items})")
    dev = torch.device(device)
    iu_val = iu_val.to(device=dev, dtype=torch.float32)
    ui_val = ui_val.to(device=dev, dtype=torch.float32)
    M_iu = Csr(iu_idx[0], iu_idx[1], num_items, num_users, dev, edge_values=iu_val)
    M_ui = Csr(ui_idx[0], ui_idx[1], num_users, num_items, dev, edge_values=ui_val)
    M_ui_T = Csr(ui_idx[1], ui_idx[0], num_items, num_users, dev, edge_values=ui_val)
    M_iu_T = Csr(iu_idx[1], iu_idx[0], num_users, num_items, dev, edge_values=iu_val)
    return OperatorPair.generic(M_iu, M_ui, M_ui_T, M_iu_T, num_users, num_items)


def square_from_torch_sparse(A: torch.Tensor, device) -> SquareOperator:
    idx, val, shape = _coo_parts(A)
    if shape[0] != shape[1]:
        raise ValueError("norm_adj must be square")
    dev = torch.device(device)
    val = val.to(device=dev, dtype=torch.float32)
    n = int(shape[0])
    return SquareOperator(Csr(idx[0], idx[1], n, n, dev, edge_values=val),
                          Csr(idx[1], idx[0], n, n, dev, edge_values=val))


def resolve_pair(item_from_user, user_from_item, num_users: int, num_items: int,
                 device=None) -> OperatorPair:
    """The OperatorPair behind two operators given in either form."""
    if isinstance(item_from_user, BipartiteOperator) and isinstance(user_from_item,
                                                                    BipartiteOperator):
        if item_from_user.pair is not user_from_item.pair:
            raise ValueError("the two operators come from different build_* calls")
        if item_from_user.role != ITEM_FROM_USER or user_from_item.role != USER_FROM_ITEM:
            raise ValueError("operator roles swapped (item<-user must be [I,U])")
        return item_from_user.pair
    if device is None:
        device = item_from_user.device
    return pair_from_torch_sparse(item_from_user, user_from_item, num_users, num_items, device)


def to_device_cred(cred_u, num_users: int, device) -> torch.Tensor | None:
    if cred_u is None:
        return None
    if isinstance(cred_u, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(cred_u.astype(np.float32, copy=False)))
    else:
        t = torch.as_tensor(cred_u)
    t = t.detach().reshape(-1).to(device=device, dtype=torch.float32).contiguous()
    if t.numel() != num_users:
        raise ValueError(f"cred vector has {t.numel()} entries, expected {num_users}")
    return t
