"""Fused BPR loss (gather -> dot -> log-sigmoid -> +reg, +fair) on the GPU.

Replaces LightGCN.bpr_loss (Version-2/lighgcn_cu_pop.py:495-508; lightgcn.py:
333-349 with the ego offset; lightgcn_cu.py:635-648 with L_fair) and its
autograd backward (index gathers + scatter-add into dense grads) with one
kernel each way (bbgr_bpr) plus a fixed-order reduction (bbgr_bpr_reduce).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import call, ld, ptr, stream_handle


def _idx(t: torch.Tensor, device) -> torch.Tensor:
    t = torch.as_tensor(t)
    return t.to(device=device, dtype=torch.int64).contiguous()


def bpr_args(users, pos, neg, uf, itf, ue, ie, reg, pop=None, lambda_fair=0.0,
             parts=None, dloss=None, g_uf=None, g_if=None, g_ue=None, g_ie=None,
             contrib=None, scores_out=None, scores=None):
    a = _lib.BprArgs()
    a.batch, a.d = users.numel(), uf.shape[1]
    a.n_users, a.n_items = uf.shape[0], itf.shape[0]
    if ue is not None and ue.shape[0] != uf.shape[0] or ie is not None and ie.shape[0] != itf.shape[0]:
        raise ValueError("ego and final tables must have the same number of rows")
    a.users, a.pos, a.neg = ptr(users), ptr(pos), ptr(neg)
    a.uf, a.lduf = ptr(uf), ld(uf)
    a.itf, a.ldif = ptr(itf), ld(itf)
    a.ue, a.ldue = ptr(ue), ld(ue)
    a.ie, a.ldie = ptr(ie), ld(ie)
    a.pop = ptr(pop)
    a.reg, a.lambda_fair = float(reg), float(lambda_fair)
    a.parts, a.dloss = ptr(parts), ptr(dloss)
    a.g_uf, a.ldguf = ptr(g_uf), ld(g_uf)
    a.g_if, a.ldgif = ptr(g_if), ld(g_if)
    a.g_ue, a.ldgue = ptr(g_ue), ld(g_ue)
    a.g_ie, a.ldgie = ptr(g_ie), ld(g_ie)
    a.contrib, a.ldcontrib = ptr(contrib), ld(contrib)
    a.scores_out, a.scores = ptr(scores_out), ptr(scores)
    return a


def bpr_loss_value(users, pos, neg, uf, itf, ue, ie, reg, pop=None, lambda_fair=0.0,
                   parts=None, out=None):
    """Loss as a 0-d device tensor (no autograd)."""
    B = users.numel()
    if B == 0:
        raise ValueError("empty batch")
    parts = torch.empty(3 * B, dtype=torch.float32, device=uf.device) if parts is None else parts
    out = torch.empty((), dtype=torch.float32, device=uf.device) if out is None else out
    a = bpr_args(users, pos, neg, uf, itf, ue, ie, reg, pop, lambda_fair, parts=parts)
    st = stream_handle()
    call("bbgr_bpr", ctypes.byref(a), st)
    call("bbgr_bpr_reduce", B, ptr(parts), float(reg), float(lambda_fair), ptr(out), st)
    return out


def _receives_dense_grad(final: torch.Tensor, weight: torch.Tensor) -> bool:
    """True when `final` is an output of the drop-in's propagate op
    (bbgr::propagate, whose backward returns a dense table) and that node hands
    `weight` (a leaf) its gradient directly. Any other node — an Add, an
    nn.Embedding(sparse=True) lookup — may return a sparse gradient, which with
    the sparse ego rows would leave .grad sparse: not accepted.
    Eager autograd only: not while compiling (dynamo traces this function) nor
    while a CUDA graph is being captured."""
    if torch.compiler.is_compiling() or not torch.is_grad_enabled():
        return False
    plain = (torch.Tensor, torch.nn.Parameter)   # not a fake / functional tensor
    if type(final) not in plain or type(weight) not in plain:
        return False
    if not weight.requires_grad or weight.grad_fn is not None:
        return False
    if weight.is_cuda and torch.cuda.is_current_stream_capturing():
        return False
    fn = final.grad_fn
    if fn is None or not _from_propagate_op(final):
        return False
    return any(nf is not None and getattr(nf, "variable", None) is weight
               for nf, _ in fn.next_functions)


def _first_slot(ids: torch.Tensor) -> torch.Tensor:
    """slot[b] = position of the first occurrence of ids[b] (device-only, fixed
    shape: stable sort, each sorted value's first sorted position by a lower-
    bound search)."""
    srt, perm = torch.sort(ids, stable=True)
    head = torch.searchsorted(srt, srt)   # first sorted position of each value
    slot = torch.empty_like(perm)
    slot[perm] = perm[head]
    return slot


# autograd nodes whose backward returns dense gradients for their leaf inputs
# and takes a sparse dL/d(u_final) (bbgr::propagate_backward_rows): the C++
# bbgr::propagate node (ops.PROPAGATE_NODE)
PROPAGATE_NODES = {"torch::autograd::CppNode<bbgr_torch::PropagateFn>",
                   "torch::autograd::CppNode<bbgr_torch::PropagateRowsFn>"}


def _from_propagate_op(final: torch.Tensor) -> bool:
    """`final` is an output of bbgr::propagate itself."""
    fn = final.grad_fn
    return fn is not None and (fn.name() in PROPAGATE_NODES
                               or type(fn).__name__ in PROPAGATE_NODES)


def ego_grad_rows(dloss, users, pos, neg, ue, ie, reg):
    """The ego-L2 gradient as compact rows: ([B, d] user rows, [2B, d]
    pos-then-neg item rows) and their table row ids, for a sparse COO
    gradient. Every occurrence of a row adds into the row of its FIRST
    occurrence, the others stay +0.0, so each table row's sum is formed exactly
    as in the dense path (the bbgr_bpr kernel's own atomics of the identical
    per-occurrence values 2·reg·dloss/B · e, computed in-kernel: one launch over
    the gathered ego rows with slot indices). A triple the kernel drops (an id
    out of range, e.g. the sampler's -1) adds nothing, as in the dense path."""
    B, d = users.numel(), ue.shape[1]
    U, I = ue.shape[0], ie.shape[0]
    valid = (users >= 0) & (users < U) & (pos >= 0) & (pos < I) & (neg >= 0) & (neg < I)
    iu = users.clamp(0, U - 1)
    ii = torch.cat([pos, neg]).clamp(0, I - 1)
    su, si = _first_slot(iu), _first_slot(ii)
    ue_c = ue.index_select(0, iu)
    ie_c = ie.index_select(0, ii)
    cu = torch.where(valid, su, -1)
    gu = torch.zeros(B, d, dtype=torch.float32, device=ue.device)
    gi = torch.zeros(2 * B, d, dtype=torch.float32, device=ue.device)
    a = bpr_args(cu, si[:B], si[B:], ue_c, ie_c, ue_c, ie_c, reg, None, 0.0,
                 dloss=dloss, g_ue=gu, g_ie=gi)
    call("bbgr_bpr", ctypes.byref(a), stream_handle())
    return gu, gi, iu, ii


def bpr_loss(users, pos_items, neg_items, user_final, item_final, user_ego, item_ego,
             reg_weight: float, pop: torch.Tensor | None = None, lambda_fair: float = 0.0):
    """Differentiable fused BPR loss (0-d tensor): the registered operator
    bbgr::bpr_loss (ops.py), backward bbgr::bpr_loss_backward.

    When the final tables come straight out of a node that already returns a
    dense gradient for the ego tables (the drop-in's propagate op, eager mode),
    the ego-L2 gradient is handed back as a sparse COO tensor of the batch rows
    (bbgr::bpr_loss_sparse_ego, as nn.Embedding(sparse=True) does): autograd
    adds it into propagate's dense table in place, so no zero-filled ego table
    is written and no dense table sum runs. `.grad` stays dense."""
    dev = user_final.device
    users, pos_items, neg_items = (_idx(t, dev) for t in (users, pos_items, neg_items))
    if not (users.numel() == pos_items.numel() == neg_items.numel()):
        raise ValueError("users, pos_items, neg_items must have equal length")
    from . import ops
    args = (user_final, item_final, user_ego, item_ego, users, pos_items, neg_items,
            float(reg_weight), pop, float(lambda_fair))
    if (_receives_dense_grad(user_final, user_ego)
            and _receives_dense_grad(item_final, item_ego)):
        return ops.bpr_loss_sparse_ego(*args, True)
    return ops.bpr_loss(*args)
