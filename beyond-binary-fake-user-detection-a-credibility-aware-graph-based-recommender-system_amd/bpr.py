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


def bpr_loss(users, pos_items, neg_items, user_final, item_final, user_ego, item_ego,
             reg_weight: float, pop: torch.Tensor | None = None, lambda_fair: float = 0.0):
    """Differentiable fused BPR loss (0-d tensor): the registered operator
    bbgr::bpr_loss (ops.py), backward bbgr::bpr_loss_backward."""
    dev = user_final.device
    users, pos_items, neg_items = (_idx(t, dev) for t in (users, pos_items, neg_items))
    if not (users.numel() == pos_items.numel() == neg_items.numel()):
        raise ValueError("users, pos_items, neg_items must have equal length")
    from . import ops
    return ops.bpr_loss(user_final, item_final, user_ego, item_ego, users, pos_items,
                        neg_items, float(reg_weight), pop, float(lambda_fair))
