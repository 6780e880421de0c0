"""The hot-path kernels as registered torch operators (torch.library).

`LightGCN.propagate()` and `LightGCN.bpr_loss()` of the drop-in modules
(Version-2/lighgcn_cu_pop.py:472-508, lightgcn_cu.py:420-463, lightgcn.py:
318-349) call these instead of Python autograd.Functions, so the drop-in step
(:858-863 — propagate, bpr_loss, backward, Adam) survives torch.compile
(dynamo traces the ops through their fake kernels, AOTAutograd sees their
registered backward) and CUDA-graph capture (the ops issue device work only,
on torch's current stream).

  bbgr::propagate(u0, i0, pair_key, num_layers, order) -> (u_final, i_final)
  bbgr::propagate_backward(gU, gI, pair_key, num_layers, order) -> (grad_u0, grad_i0)
  bbgr::jacobi_layer(u, i, pair_key) -> (new_i, new_u)   (+ _backward)
  bbgr::propagate_sym(x0, pair_key, num_layers) -> x_final   (+ _backward)
  bbgr::bpr_loss(uf, itf, ue, ie, users, pos, neg, reg, pop, lambda_fair) -> loss
  bbgr::bpr_loss_backward(dloss, uf, itf, ue, ie, users, pos, neg, reg, pop,
                          lambda_fair) -> (g_uf, g_if, g_ue, g_ie)
  bbgr::bpr_loss_sparse_ego(..., sparse_uf) -> loss   (eager drop-in step: the
      ego gradients, and with sparse_uf dL/d(u_final), go back as sparse rows)
  bbgr::propagate_backward_rows(iu, vu, gI, num_users, pair_key, num_layers,
                                order) -> (grad_u0, grad_i0)   (gU given as rows)

The sparse operators are not tensors: an OperatorPair is registered once
(`pair_key`) and the ops look it up; shapes for the fake kernels come from
the tensor arguments alone.
"""
from __future__ import annotations

import ctypes
import itertools
import weakref
from typing import Optional

import torch
from torch import Tensor
from torch.library import custom_op

from . import _lib
from ._lib import call, stream_handle

# key -> OperatorPair, held weakly: the model that owns a pair keeps it (and
# its device CSRs) alive, the registry does not
_PAIRS: "weakref.WeakValueDictionary[int, object]" = weakref.WeakValueDictionary()
_keys = itertools.count(1)


def pair_key(pair) -> int:
    """The registry key of an OperatorPair (assigned on first use)."""
    k = getattr(pair, "_op_key", None)
    if k is None:
        k = next(_keys)
        pair._op_key = k
        _PAIRS[k] = pair
    return k


def _pair(key: int):
    try:
        return _PAIRS[key]
    except KeyError:
        raise RuntimeError(f"bbgr ops: no operator pair registered under key {key}") from None


# -- propagation -------------------------------------------------------------
@custom_op("bbgr::propagate", mutates_args=())
def propagate(u0: Tensor, i0: Tensor, pair_key: int, num_layers: int,
              order: str) -> tuple[Tensor, Tensor]:
    from .propagate import forward
    _lib.require_gpu(u0)
    return forward(_pair(pair_key), u0.contiguous(), i0.contiguous(), num_layers, order)


@propagate.register_fake
def _(u0, i0, pair_key, num_layers, order):
    return u0.new_empty(u0.shape), i0.new_empty(i0.shape)


def grad_support(pair, gU: Tensor, gI: Tensor, order: str):
    """(user mask, item mask) for propagate.backward's grad_support, read off
    the gradients themselves (bbgr_row_support, one pass over each table): the
    users with a nonzero gU row; the items with a nonzero gI row, plus for GS
    every neighbour of a flagged user (the first item product's output
    support). A BPR loss touches only the batch rows, so the first backward
    products then skip all but those rows — bitwise the dense chain's result
    (a skipped row is exactly zero)."""
    from .propagate import ORDER_GS
    st = stream_handle()
    U, I = pair.num_users, pair.num_items
    mu = torch.empty(max(U, 1), dtype=torch.uint8, device=gU.device)
    mi = torch.empty(max(I, 1), dtype=torch.uint8, device=gU.device)
    d = gU.shape[1]
    call("bbgr_row_support", I, d, _lib.ptr(gI), _lib.ld(gI), _lib.ptr(mi), None, None, None, st)
    if pair.io is not None:   # input-order tables over a degree-ordered graph
        call("bbgr_row_support", U, d, _lib.ptr(gU), _lib.ld(gU), _lib.ptr(mu), None, None,
             None, st)
        return _io_support(pair, mu[:U], mi[:I], order)
    uc = pair.fwd_user.csr if order == ORDER_GS else None   # user rows -> item neighbours
    call("bbgr_row_support", U, d, _lib.ptr(gU), _lib.ld(gU), _lib.ptr(mu),
         None if uc is None else _lib.ptr(uc.indptr),
         None if uc is None else _lib.ptr(uc.indices),
         None if uc is None else _lib.ptr(mi), st)
    return mu[:U], mi[:I]


def _io_support(pair, mu: Tensor, mi: Tensor, order: str, users: Optional[Tensor] = None):
    """grad_support of an input-order pair (propagate.backward_steps): (user mask,
    item mask) in the caller's input order plus the item mask in the graph's
    internal order (the first item product's row mask); GS adds the item
    neighbours of every flagged user (of `users`, input ids, when given) to both
    item masks."""
    from .propagate import ORDER_GS
    io = pair.io
    if order != ORDER_GS:
        return mu, mi, None
    st = stream_handle()
    mi_int = mi[io.item_map64]
    uc = pair.fwd_user.csr
    if users is not None:
        ui = io.user_rank64[users]
        call("bbgr_mark_neighbors", ui.numel(), _lib.ptr(ui), _lib.ptr(uc.indptr),
             _lib.ptr(uc.indices), 1, _lib.ptr(mi_int), st)
    else:
        call("bbgr_mark_neighbors_of_mask", pair.num_users, _lib.ptr(mu), _lib.ptr(io.user_map),
             _lib.ptr(uc.indptr), _lib.ptr(uc.indices), 1, _lib.ptr(mi_int), st)
    return mu, mi_int[io.item_rank64], mi_int


@custom_op("bbgr::propagate_backward", mutates_args=())
def propagate_backward(gU: Tensor, gI: Tensor, pair_key: int, num_layers: int,
                       order: str) -> tuple[Tensor, Tensor]:
    from .propagate import backward
    _lib.require_gpu(gU)
    pair = _pair(pair_key)
    gU, gI = gU.contiguous(), gI.contiguous()
    return backward(pair, gU, gI, num_layers, order,
                    grad_support=grad_support(pair, gU, gI, order))


@propagate_backward.register_fake
def _(gU, gI, pair_key, num_layers, order):
    return gU.new_empty(gU.shape), gI.new_empty(gI.shape)


def _propagate_setup(ctx, inputs, output):
    u0, i0, ctx.key, ctx.K, ctx.order = inputs
    ctx.shapes = (u0.shape, i0.shape)


@custom_op("bbgr::propagate_backward_rows", mutates_args=())
def propagate_backward_rows(iu: Tensor, vu: Tensor, gI: Tensor, num_users: int, pair_key: int,
                            num_layers: int, order: str) -> tuple[Tensor, Tensor]:
    """propagate_backward with dL/d(u_final) given as rows: vu[k] adds to user
    iu[k] (a sparse COO gradient's indices and values, e.g. a BPR batch). The
    dense gU is formed on the listed rows only (zeroed, then the rows summed in
    ascending k — bbgr_scatter_add_rows, as the dense BPR backward forms them)
    and the masks come from the list (bbgr_mark_rows / bbgr_mark_neighbors)
    instead of a pass over a zero-filled table: every read of gU in the
    backward chain is masked to those rows, so the rest is never touched.
    The masks are a superset of the value-derived ones: bitwise the same."""
    from .propagate import ORDER_GS, backward
    from .scatter import index_add_rows
    _lib.require_gpu(vu)
    pair = _pair(pair_key)
    U, I, d = pair.num_users, pair.num_items, vu.shape[1]
    if num_users != U:
        raise ValueError("propagate_backward_rows: num_users does not match the operator pair")
    st = stream_handle()
    iu = iu.to(torch.int64).contiguous()
    gI = gI.contiguous()
    if num_layers == 0:   # K = 0: backward copies gU whole (grad_u0 = gU), so no
        # row may stay uninitialised
        gU = torch.zeros(max(U, 1), d, dtype=torch.float32, device=vu.device)[:U]
    else:   # every read of gU in the K >= 1 chain is masked to the listed rows
        gU = torch.empty(max(U, 1), d, dtype=torch.float32, device=vu.device)[:U]
        gU.index_fill_(0, iu, 0.0)
    index_add_rows(gU, iu, vu.contiguous())
    mu = torch.zeros(max(U, 1), dtype=torch.uint8, device=vu.device)
    mi = torch.empty(max(I, 1), dtype=torch.uint8, device=vu.device)
    call("bbgr_mark_rows", iu.numel(), _lib.ptr(iu), 1, _lib.ptr(mu), U, st)
    call("bbgr_row_support", I, d, _lib.ptr(gI), _lib.ld(gI), _lib.ptr(mi), None, None, None, st)
    if pair.io is not None:   # input-order tables over a degree-ordered graph
        return backward(pair, gU, gI, num_layers, order,
                        grad_support=_io_support(pair, mu[:U], mi[:I], order, users=iu))
    if order == ORDER_GS:   # the first item product's output support: N(listed users)
        uc = pair.fwd_user.csr
        call("bbgr_mark_neighbors", iu.numel(), _lib.ptr(iu), _lib.ptr(uc.indptr),
             _lib.ptr(uc.indices), 1, _lib.ptr(mi), st)
    return backward(pair, gU, gI, num_layers, order, grad_support=(mu[:U], mi[:I]))


@propagate_backward_rows.register_fake
def _(iu, vu, gI, num_users, pair_key, num_layers, order):
    return vu.new_empty((num_users, vu.shape[1])), gI.new_empty(gI.shape)


def _propagate_bwd(ctx, gU, gI):
    (su, si) = ctx.shapes
    if gU is not None and gU.layout == torch.sparse_coo and (gI is None or not gI.is_sparse):
        # BPR-shaped gradient handed over as rows (bbgr::bpr_loss_sparse_ego)
        gI = gU._values().new_zeros(si) if gI is None else gI
        gu0, gi0 = propagate_backward_rows(gU._indices()[0], gU._values(), gI, su[0],
                                           ctx.key, ctx.K, ctx.order)
        return gu0, gi0, None, None, None
    if gU is not None and gU.is_sparse:
        gU = gU.to_dense()
    if gI is not None and gI.is_sparse:
        gI = gI.to_dense()
    ref = gU if gU is not None else gI
    if gU is None:
        gU = ref.new_zeros(su)
    if gI is None:
        gI = ref.new_zeros(si)
    gu0, gi0 = propagate_backward(gU, gI, ctx.key, ctx.K, ctx.order)
    return gu0, gi0, None, None, None


propagate.register_autograd(_propagate_bwd, setup_context=_propagate_setup)


# -- one Jacobi layer (lightgcn_cu.py propagate_all_layers, :420-448) ------------
@custom_op("bbgr::jacobi_layer", mutates_args=())
def jacobi_layer(u: Tensor, i: Tensor, pair_key: int) -> tuple[Tensor, Tensor]:
    from .propagate import spmm
    _lib.require_gpu(u)
    pair = _pair(pair_key)
    u, i = u.contiguous(), i.contiguous()
    FI, FU = pair.fwd_item, pair.fwd_user
    new_i = torch.empty(pair.num_items, u.shape[1], device=u.device)
    new_u = torch.empty(pair.num_users, u.shape[1], device=u.device)
    io = pair.io   # input-order layer tables: input-id gathers, mapped output rows
    spmm(FI, u, True, y=new_i, y_scale=FI.out_scale, src_input=io is not None,
         y_map=None if io is None else io.item_map)
    spmm(FU, i, True, y=new_u, y_scale=FU.out_scale, src_input=io is not None,
         y_map=None if io is None else io.user_map)
    return new_i, new_u


@jacobi_layer.register_fake
def _(u, i, pair_key):
    return i.new_empty(i.shape), u.new_empty(u.shape)


@custom_op("bbgr::jacobi_layer_backward", mutates_args=())
def jacobi_layer_backward(g_i: Tensor, g_u: Tensor, pair_key: int) -> tuple[Tensor, Tensor]:
    """(d/du, d/di): M_iu^T g_i on the user rows, M_ui^T g_u on the item rows."""
    from .propagate import spmm
    pair = _pair(pair_key)
    BI, BU = pair.bwd_item, pair.bwd_user
    gu = torch.empty(pair.num_users, g_i.shape[1], device=g_i.device)
    gi = torch.empty(pair.num_items, g_u.shape[1], device=g_u.device)
    io = pair.io
    spmm(BU, g_i.contiguous(), True, y=gu, y_scale=BU.out_scale, src_input=io is not None,
         y_map=None if io is None else io.user_map)
    spmm(BI, g_u.contiguous(), True, y=gi, y_scale=BI.out_scale, src_input=io is not None,
         y_map=None if io is None else io.item_map)
    return gu, gi


@jacobi_layer_backward.register_fake
def _(g_i, g_u, pair_key):
    return g_u.new_empty(g_u.shape), g_i.new_empty(g_i.shape)


def _layer_setup(ctx, inputs, output):
    u, i, ctx.key = inputs
    ctx.shapes = (u.shape, i.shape)


def _layer_bwd(ctx, g_i, g_u):
    su, si = ctx.shapes
    ref = g_i if g_i is not None else g_u
    g_i = ref.new_zeros(si) if g_i is None else g_i
    g_u = ref.new_zeros(su) if g_u is None else g_u
    gu, gi = jacobi_layer_backward(g_i, g_u, ctx.key)
    return gu, gi, None


jacobi_layer.register_autograd(_layer_bwd, setup_context=_layer_setup)


# -- symmetric operator (lightgcn.py): one stacked [users; items] table ------------
@custom_op("bbgr::propagate_sym", mutates_args=())
def propagate_sym(x0: Tensor, pair_key: int, num_layers: int) -> Tensor:
    from .propagate import ORDER_J, forward
    _lib.require_gpu(x0)
    pair = _pair(pair_key)
    U = pair.num_users
    x0 = x0.contiguous()
    out = torch.empty_like(x0)
    forward(pair, x0[:U], x0[U:], num_layers, ORDER_J, out_u=out[:U], out_i=out[U:])
    return out


@propagate_sym.register_fake
def _(x0, pair_key, num_layers):
    return x0.new_empty(x0.shape)


@custom_op("bbgr::propagate_sym_backward", mutates_args=())
def propagate_sym_backward(g: Tensor, pair_key: int, num_layers: int) -> Tensor:
    from .propagate import ORDER_J, backward
    pair = _pair(pair_key)
    U = pair.num_users
    g = g.contiguous()
    gx = torch.empty_like(g)
    backward(pair, g[:U], g[U:], num_layers, ORDER_J, out_u=gx[:U], out_i=gx[U:],
             grad_support=grad_support(pair, g[:U], g[U:], ORDER_J))
    return gx


@propagate_sym_backward.register_fake
def _(g, pair_key, num_layers):
    return g.new_empty(g.shape)


def _sym_setup(ctx, inputs, output):
    _, ctx.key, ctx.K = inputs


def _sym_bwd(ctx, g):
    return propagate_sym_backward(g, ctx.key, ctx.K), None, None


propagate_sym.register_autograd(_sym_bwd, setup_context=_sym_setup)


# -- BPR loss ------------------------------------------------------------------
@custom_op("bbgr::bpr_loss", mutates_args=())
def bpr_loss(uf: Tensor, itf: Tensor, ue: Tensor, ie: Tensor, users: Tensor, pos: Tensor,
             neg: Tensor, reg: float, pop: Optional[Tensor], lambda_fair: float) -> Tensor:
    from .bpr import bpr_loss_value
    _lib.require_gpu(uf)
    return bpr_loss_value(users, pos, neg, uf.contiguous(), itf.contiguous(), ue.contiguous(),
                          ie.contiguous(), reg, pop, lambda_fair)


@bpr_loss.register_fake
def _(uf, itf, ue, ie, users, pos, neg, reg, pop, lambda_fair):
    return uf.new_empty(())


@custom_op("bbgr::bpr_loss_backward", mutates_args=())
def bpr_loss_backward(dloss: Tensor, uf: Tensor, itf: Tensor, ue: Tensor, ie: Tensor,
                      users: Tensor, pos: Tensor, neg: Tensor, reg: float,
                      pop: Optional[Tensor], lambda_fair: float
                      ) -> tuple[Tensor, Tensor, Tensor, Tensor]:
    """Deterministic: the kernel writes per-triple gradient rows of the final
    tables (contrib) and bbgr_scatter_add_rows sums each destination's rows in
    ascending triple order; the ego-L2 rows add one identical value per
    occurrence, whose order cannot change the sum."""
    from .bpr import bpr_args
    from .scatter import index_add_rows
    uf, itf, ue, ie = (t.contiguous() for t in (uf, itf, ue, ie))
    g_uf, g_if, g_ue, g_ie = (torch.zeros_like(t) for t in (uf, itf, ue, ie))
    B = users.numel()
    contrib = torch.empty(3 * B, uf.shape[1], dtype=torch.float32, device=uf.device)
    d = dloss.to(torch.float32).contiguous().reshape(())
    a = bpr_args(users, pos, neg, uf, itf, ue, ie, reg, pop, lambda_fair, dloss=d,
                 g_ue=g_ue, g_ie=g_ie, contrib=contrib)
    call("bbgr_bpr", ctypes.byref(a), stream_handle())
    index_add_rows(g_uf, users, contrib[:B])
    index_add_rows(g_if, torch.cat([pos, neg]), contrib[B:])
    return g_uf, g_if, g_ue, g_ie


@bpr_loss_backward.register_fake
def _(dloss, uf, itf, ue, ie, users, pos, neg, reg, pop, lambda_fair):
    return (uf.new_empty(uf.shape), itf.new_empty(itf.shape), ue.new_empty(ue.shape),
            ie.new_empty(ie.shape))


def _bpr_setup(ctx, inputs, output):
    uf, itf, ue, ie, users, pos, neg, reg, pop, lam = inputs
    ctx.save_for_backward(uf, itf, ue, ie, users, pos, neg)
    ctx.reg, ctx.lam = reg, lam
    ctx.pop = pop


def _bpr_bwd(ctx, gloss):
    uf, itf, ue, ie, users, pos, neg = ctx.saved_tensors
    g = bpr_loss_backward(gloss, uf, itf, ue, ie, users, pos, neg, ctx.reg, ctx.pop, ctx.lam)
    return g[0], g[1], g[2], g[3], None, None, None, None, None, None


bpr_loss.register_autograd(_bpr_bwd, setup_context=_bpr_setup)


# -- BPR loss, ego gradient as sparse batch rows (eager drop-in step) -------------
@custom_op("bbgr::bpr_loss_sparse_ego", mutates_args=())
def bpr_loss_sparse_ego(uf: Tensor, itf: Tensor, ue: Tensor, ie: Tensor, users: Tensor,
                        pos: Tensor, neg: Tensor, reg: float, pop: Optional[Tensor],
                        lambda_fair: float, sparse_uf: bool) -> Tensor:
    """bbgr::bpr_loss whose backward returns the ego-table gradients as sparse
    COO batch rows (bpr.bpr_loss picks it only when the final tables' node
    returns dense gradients for the same ego tables; autograd then adds the
    rows into that dense table in place). `sparse_uf` (uf is bbgr::propagate's
    output): dL/d(uf) goes back as sparse batch rows too, which propagate's
    backward consumes without a zero-filled table (propagate_backward_rows)."""
    from .bpr import bpr_loss_value
    _lib.require_gpu(uf)
    return bpr_loss_value(users, pos, neg, uf.contiguous(), itf.contiguous(), ue.contiguous(),
                          ie.contiguous(), reg, pop, lambda_fair)


@bpr_loss_sparse_ego.register_fake
def _(uf, itf, ue, ie, users, pos, neg, reg, pop, lambda_fair, sparse_uf):
    return uf.new_empty(())


def _bpr_se_setup(ctx, inputs, output):
    _bpr_setup(ctx, inputs[:10], output)
    ctx.sparse_uf = inputs[10]


def _bpr_se_bwd(ctx, gloss):
    from .bpr import bpr_args, ego_grad_rows
    from .scatter import index_add_rows
    uf, itf, ue, ie, users, pos, neg = ctx.saved_tensors
    uf, itf, ue, ie = (t.contiguous() for t in (uf, itf, ue, ie))
    B = users.numel()
    d = gloss.to(torch.float32).contiguous().reshape(())
    contrib = torch.empty(3 * B, uf.shape[1], dtype=torch.float32, device=uf.device)
    a = bpr_args(users, pos, neg, uf, itf, ue, ie, ctx.reg, ctx.pop, ctx.lam, dloss=d,
                 contrib=contrib)
    call("bbgr_bpr", ctypes.byref(a), stream_handle())
    g_if = torch.zeros_like(itf)
    index_add_rows(g_if, torch.cat([pos, neg]), contrib[B:])
    ru, ri, iu, ii = ego_grad_rows(d, users, pos, neg, ue, ie, ctx.reg)
    if ctx.sparse_uf:   # rows for bbgr::propagate's backward (propagate_backward_rows);
        # a dropped triple's row is +0.0 (the kernel zeroes it), so clamped ids add nothing
        g_uf = torch.sparse_coo_tensor(iu.unsqueeze(0), contrib[:B], uf.shape)
    else:
        g_uf = torch.zeros_like(uf)
        index_add_rows(g_uf, users, contrib[:B])
    g_ue = torch.sparse_coo_tensor(iu.unsqueeze(0), ru, ue.shape)
    g_ie = torch.sparse_coo_tensor(ii.unsqueeze(0), ri, ie.shape)
    return g_uf, g_if, g_ue, g_ie, None, None, None, None, None, None, None


bpr_loss_sparse_ego.register_autograd(_bpr_se_bwd, setup_context=_bpr_se_setup)
