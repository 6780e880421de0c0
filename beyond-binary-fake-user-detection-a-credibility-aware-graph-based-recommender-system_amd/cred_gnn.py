"""Credibility GNN aggregation on the device.

Drop-in for the ``CredModel`` defined inside ``train_and_export_credibility``
(main.py:659-707): same sub-modules and state_dict keys (``user_proj``,
``item_proj``, ``item_upd``, ``user_upd``, ``out``), same methods
(``ewa_raw``, ``normalize_per_dst``, ``aggregate``, ``forward_subgraph``) and
return values. The linear layers stay torch GEMMs (library GEMMs); the
edge-wise work — EWA weights (Eq. 3.12), per-destination normalisation and the
two weighted ``index_add_`` aggregations (Eq. 3.13-3.16) — runs as:

* one destination-row CSR and one source-row CSR per subgraph direction,
  built on the device (``bbgr_csr_build``, with the edge permutation);
* ``bbgr_ewa_normalize``: raw weights (one gather into CSR order),
  fixed-order per-destination sums and the normalised weights in CSR and
  input order (coalesced passes);
* the aggregation = ``bbgr_spmm`` over the destination CSR with the
  normalised weights as edge values; its gradient w.r.t. the source features
  = ``bbgr_spmm`` over the source CSR (the transpose). No atomics: the
  aggregation and its backward are bitwise deterministic, where the
  reference's ``index_add_`` on a GPU is not.

Edge weights come from edge attributes (no gradient), as in the reference.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from ._lib import call, ptr, stream_handle
from .graph import Csr
from .propagate import Product, spmm

EDGE_ATTR_KEYS = ["verified", "rating_align", "rating", "timestamp_norm", "helpful_vote"]  # main.py:71
BETA = 1.0    # main.py:626 (EWA, Eq. 3.12)
GAMMA = 1.0   # main.py:627
NORM_EPS = 1e-12   # main.py:684


class EdgeSet:
    """Edges src -> dst of one subgraph direction, indexed both ways on the
    device. ``edge_index``: [2, E] (row 0 = source, row 1 = destination)."""

    def __init__(self, edge_index: torch.Tensor, num_src: int, num_dst: int, device=None):
        device = torch.device(device if device is not None else edge_index.device)
        _lib.require_gpu()
        ei = torch.as_tensor(edge_index)
        self.num_src, self.num_dst = int(num_src), int(num_dst)
        self.E = int(ei.shape[1])
        src, dst = ei[0].to(device), ei[1].to(device)
        self.by_dst = Csr(dst, src, num_dst, num_src, device, keep_perm=True)
        self.by_src = Csr(src, dst, num_src, num_dst, device, keep_perm=True)
        # each edge's destination row (input order): w~ in input order is then
        # one coalesced pass instead of a scatter through the CSR permutation
        self.dst = dst.to(torch.int32).contiguous()
        self.device = device

    def normalize(self, w: torch.Tensor | None = None, edge_attr: torch.Tensor | None = None,
                  col_verified: int = 0, col_align: int = 1, beta: float = BETA,
                  gamma: float = GAMMA, eps: float = NORM_EPS):
        """(w_raw, w_tilde) in input-edge order and the normalised weights in
        destination-CSR order (the aggregation's edge values). Either raw
        weights `w` (normalize_per_dst) or `edge_attr` (EWA, then normalise)."""
        E = self.E
        f32 = dict(dtype=torch.float32, device=self.device)
        w_raw = torch.empty(max(E, 1), **f32)
        w_edge = torch.empty(max(E, 1), **f32)
        w_csr = torch.empty(max(E, 1), **f32)
        if E:
            if w is not None:
                w_in = w.detach().to(**f32).contiguous()
                attr, lda = None, 0
            else:
                w_in = None
                attr = edge_attr.detach().to(**f32).contiguous()
                lda = attr.shape[1]
            cs = self.by_dst.struct()
            args = (ctypes.byref(cs), ptr(self.by_dst.perm), ptr(self.dst), ptr(w_in), ptr(attr), lda,
                    col_verified, col_align, float(beta), float(gamma), float(eps), ptr(w_raw),
                    ptr(w_edge), ptr(w_csr))
            n = ctypes.c_size_t(0)
            call("bbgr_ewa_normalize", *args, None, ctypes.byref(n), stream_handle())
            ws = torch.empty(max(n.value, 1), dtype=torch.uint8, device=self.device)
            call("bbgr_ewa_normalize", *args, ptr(ws), ctypes.byref(n), stream_handle())
        return w_raw[:E], w_edge[:E], w_csr[:E]

    def src_order(self, w_edge: torch.Tensor) -> torch.Tensor:
        """Per-edge values permuted into source-CSR order (the transpose)."""
        if self.E == 0:
            return w_edge
        return w_edge[self.by_src.perm[: self.E].long()].contiguous()


class _AggregateFn(torch.autograd.Function):
    """out[dst] = sum_e w_e * x[src_e]; d out / d x = the transposed product."""

    @staticmethod
    def forward(ctx, x, edges: EdgeSet, w_csr, w_src):
        x = x.contiguous()
        out = torch.empty(edges.num_dst, x.shape[1], dtype=torch.float32, device=x.device)
        if edges.E == 0:
            out.zero_()
        else:
            spmm(Product(edges.by_dst, w_csr, None, None, {}), x, False, y=out)
        ctx.edges, ctx.w_src = edges, w_src
        return out

    @staticmethod
    def backward(ctx, g):
        edges = ctx.edges
        g = g.contiguous()
        gx = torch.empty(edges.num_src, g.shape[1], dtype=torch.float32, device=g.device)
        if edges.E == 0:
            gx.zero_()
        else:
            spmm(Product(edges.by_src, ctx.w_src, None, None, {}), g, False, y=gx)
        return gx, None, None, None


def aggregate(src_x: torch.Tensor, edges: EdgeSet, w_edge: torch.Tensor,
              w_csr: torch.Tensor | None = None) -> torch.Tensor:
    """CredModel.aggregate (main.py:687-691) over a prepared EdgeSet."""
    _lib.require_gpu(src_x)
    if src_x.dtype != torch.float32 or src_x.shape[1] not in (64, 128, 256):
        raise ValueError("aggregate: fp32 features of width 64, 128 or 256")
    if w_csr is None:   # weights given in input order: permute to dst-CSR order
        w_csr = (w_edge[edges.by_dst.perm[: edges.E].long()].contiguous()
                 if edges.E else w_edge)
    return _AggregateFn.apply(src_x, edges, w_csr, edges.src_order(w_edge))


class CredModel(nn.Module):
    """main.py:659-707, GraphSAGE-style two-stage aggregation with EWA weights."""

    def __init__(self, user_in_dim, item_in_dim, hidden_dim, edge_attr_keys=EDGE_ATTR_KEYS,
                 beta: float = BETA, gamma: float = GAMMA):
        super().__init__()
        self.user_proj = nn.Linear(user_in_dim, hidden_dim)
        self.item_proj = nn.Linear(item_in_dim, hidden_dim)
        self.item_upd = nn.Linear(hidden_dim * 2, hidden_dim)
        self.user_upd = nn.Linear(hidden_dim * 2, hidden_dim)
        self.out = nn.Linear(hidden_dim, 1)
        self.edge_attr_keys = edge_attr_keys
        self.EDGE_VERIFIED = edge_attr_keys.index("verified")
        self.EDGE_ALIGN = edge_attr_keys.index("rating_align")
        self.beta, self.gamma = beta, gamma

    # -- the reference's helpers, on the device ---------------------------------
    def ewa_raw(self, edge_attr: torch.Tensor) -> torch.Tensor:
        """w = clamp(beta*clamp(verified,0,1) + gamma*rating_align, min=0) (:677-681)."""
        E = edge_attr.shape[0]
        idx = torch.arange(E, dtype=torch.int64, device=edge_attr.device)
        es = EdgeSet(torch.stack([idx, idx]), E, E)   # identity: one edge per row
        w_raw, _, _ = es.normalize(edge_attr=edge_attr, col_verified=self.EDGE_VERIFIED,
                                   col_align=self.EDGE_ALIGN, beta=self.beta, gamma=self.gamma)
        return w_raw

    def normalize_per_dst(self, w: torch.Tensor, dst: torch.Tensor, num_dst: int) -> torch.Tensor:
        """w / (scatter_add(w, dst) + 1e-12)[dst] (:683-685)."""
        E = w.shape[0]
        src = torch.zeros(E, dtype=torch.int64, device=w.device)
        es = EdgeSet(torch.stack([src, dst.to(w.device)]), 1, num_dst)
        _, w_edge, _ = es.normalize(w=w)
        return w_edge

    def aggregate(self, src_x: torch.Tensor, edge_index: torch.Tensor, w_tilde: torch.Tensor,
                  num_dst: int) -> torch.Tensor:
        """scatter_add(w_tilde * src_x[src], dst) (:687-691)."""
        es = EdgeSet(edge_index, src_x.shape[0], num_dst)
        return aggregate(src_x, es, w_tilde)

    # -- the fused subgraph forward ---------------------------------------------
    def forward_subgraph(self, x_u, x_i, e_u2i, ea_u2i, e_i2u, ea_i2u):
        """(cred, h_u2, h_i1, w1t) of main.py:693-707. Each direction's CSRs are
        built once and serve the weights, the aggregation and its backward."""
        h_u0 = self.user_proj(x_u)
        h_i0 = self.item_proj(x_i)
        nu, ni = h_u0.shape[0], h_i0.shape[0]
        cols = dict(col_verified=self.EDGE_VERIFIED, col_align=self.EDGE_ALIGN,
                    beta=self.beta, gamma=self.gamma)

        s1 = EdgeSet(e_u2i, nu, ni)
        _, w1t, w1c = s1.normalize(edge_attr=ea_u2i, **cols)
        m_i1 = aggregate(h_u0, s1, w1t, w1c)
        h_i1 = F.relu(self.item_upd(torch.cat([h_i0, m_i1], dim=-1)))

        s2 = EdgeSet(e_i2u, ni, nu)
        _, w2t, w2c = s2.normalize(edge_attr=ea_i2u, **cols)
        m_u2 = aggregate(h_i1, s2, w2t, w2c)
        h_u2 = F.relu(self.user_upd(torch.cat([h_u0, m_u2], dim=-1)))

        cred = torch.sigmoid(self.out(h_u2)).squeeze(-1)
        return cred, h_u2, h_i1, w1t
