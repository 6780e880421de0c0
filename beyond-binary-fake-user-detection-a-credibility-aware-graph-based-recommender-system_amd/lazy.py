"""Deferred final tables for the drop-in LightGCN (Gauss-Seidel order).

The reference's training loop reads the propagated tables only through the
BPR loss, at the batch rows (Version-2/lighgcn_cu_pop.py:858-859):

    user_emb, item_emb = model.get_user_item_emb()
    loss = model.bpr_loss(users_t, pos_t, neg_t, user_emb, item_emb, cfg.reg)

Computing the whole (u_final, i_final) there costs the last layer's two full
products and a full-table layer-mean pass per layer (C4: ~3.7 ms of the
~11 ms forward) for values nobody reads. `propagate()` therefore returns two
DeferredFinal tensors: they carry the call's weights and compute nothing
until used.

  * `bpr_loss` handed both tables of one call computes only the batch rows
    (bbgr::propagate_rows: the dense layers 1..K-1, the last layer on the item
    frontier and the batch users). Same bits at those rows, and the same
    autograd backward as bbgr::propagate, so the loss and every gradient are
    those of the dense path.
  * ANY other use (indexing, arithmetic, .cpu(), printing, a torch op, a raw
    data_ptr) runs the dense bbgr::propagate once, under the grad mode of the
    propagate() call, and proceeds on its tables: evaluation code sees the
    reference's full tables. Shape / dtype / device queries answer without
    computing.
  * The weights must not change between propagate() and the first use (the
    reference never does that): a use after an in-place update of either
    weight raises instead of returning tables of the new weights.

Eager mode only: while compiling (torch.compile) or capturing a CUDA graph,
and on CPU tables, propagate() returns the dense tables as before. Set
`LightGCN.lazy_finals = False` (class or instance) to always compute them.
"""
from __future__ import annotations

import torch
from torch.utils._pytree import tree_map


class _Pending:
    """One propagate() call: its weights, their versions, its grad mode, and
    the dense tables once computed."""

    def __init__(self, full_fn, rows_fn, u0: torch.Tensor, i0: torch.Tensor, step=None):
        self.full_fn, self.rows_fn = full_fn, rows_fn
        self.u0, self.i0 = u0, i0
        self.step = step   # (pair_key, num_layers, row maps or None) of a GS chain: the in-backward Adam
        self.version = (u0._version, i0._version)
        self.grad = torch.is_grad_enabled()
        self.out = None

    def _check(self) -> None:
        if (self.u0._version, self.i0._version) != self.version:
            raise RuntimeError(
                "bbgr: the final tables of a propagate() call were read after the embedding "
                "weights changed in place; read them before the optimizer step, or set "
                "LightGCN.lazy_finals = False to compute them at the call")

    def full(self):
        if self.out is None:
            self._check()
            with torch.set_grad_enabled(self.grad):
                self.out = self.full_fn()
        return self.out

    def rows(self, users: torch.Tensor, items: torch.Tensor):
        self._check()
        with torch.set_grad_enabled(self.grad):
            return self.rows_fn(users, items)


# metadata the placeholder answers itself (no computation)
_META = {
    torch.Tensor.shape.__get__, torch.Tensor.dtype.__get__, torch.Tensor.device.__get__,
    torch.Tensor.layout.__get__, torch.Tensor.is_cuda.__get__, torch.Tensor.ndim.__get__,
    torch.Tensor.requires_grad.__get__, torch.Tensor.size, torch.Tensor.dim,
    torch.Tensor.numel, torch.Tensor.__len__,
}


def _resolve(x):
    return x._pending.full()[x._side] if isinstance(x, DeferredFinal) else x


class DeferredFinal(torch.Tensor):
    """One final table of a propagate() call (side 0: users, 1: items),
    computed on first use (module docstring). Its own storage is a shared
    uninitialised table of the right shape (_placeholder): nothing reads it."""

    @staticmethod
    def __new__(cls, pending: _Pending, side: int, like: torch.Tensor, requires_grad: bool):
        t = torch.Tensor._make_subclass(cls, like, requires_grad)
        t._pending, t._side = pending, side
        return t

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func in _META:
            with torch._C.DisableTorchFunctionSubclass():
                return func(*args, **kwargs)
        args, kwargs = tree_map(_resolve, (args, kwargs))
        return func(*args, **kwargs)

    def __repr__(self, *, tensor_contents=None):
        return repr(_resolve(self))


def supported(u0: torch.Tensor, i0: torch.Tensor) -> bool:
    """Deferral applies: eager mode, device tables, no graph capture."""
    if not (u0.is_cuda and i0.is_cuda) or torch.compiler.is_compiling():
        return False
    plain = (torch.Tensor, torch.nn.Parameter)
    if type(u0) not in plain or type(i0) not in plain:
        return False
    return not torch.cuda.is_current_stream_capturing()


# One placeholder table per (shape, dtype, device), shared by every deferred
# table of that shape: nothing reads or writes it (every use resolves first),
# it only gives the tensor its metadata and in-bounds storage.
_placeholders: dict = {}


def _placeholder(like: torch.Tensor) -> torch.Tensor:
    key = (tuple(like.shape), like.dtype, like.device)
    t = _placeholders.get(key)
    if t is None:
        if len(_placeholders) >= 4:   # a few model shapes alive at once, at most
            _placeholders.pop(next(iter(_placeholders)))
        t = _placeholders[key] = torch.empty(like.shape, dtype=like.dtype, device=like.device)
    return t


def deferred_pair(full_fn, rows_fn, u0: torch.Tensor, i0: torch.Tensor, step=None):
    """(u_final, i_final) as DeferredFinal tensors of one call. `step`:
    (pair_key, num_layers) when the chain is GS (fused_bpr_step may run it)."""
    p = _Pending(full_fn, rows_fn, u0, i0, step)
    rg = p.grad and (u0.requires_grad or i0.requires_grad)
    return (DeferredFinal(p, 0, _placeholder(u0.detach()), rg),
            DeferredFinal(p, 1, _placeholder(i0.detach()), rg))


def batch_finals(user_final, item_final, users, pos, neg):
    """bpr_loss's tables: (u_final, i_final, users, pos, neg) with the finals
    valid at the batch rows when both come from one deferred call (the index
    vectors as device int64), else the finals resolved (dense) and the
    indices as given."""
    if (isinstance(user_final, DeferredFinal) and isinstance(item_final, DeferredFinal)
            and user_final._pending is item_final._pending and user_final._side == 0
            and item_final._side == 1 and user_final._pending.out is None):
        p = user_final._pending
        dev = p.u0.device
        users, pos, neg = (torch.as_tensor(t).to(device=dev, dtype=torch.int64).contiguous()
                           for t in (users, pos, neg))
        uf, itf = p.rows(users, torch.cat([pos, neg]))
        return uf, itf, users, pos, neg
    return _resolve(user_final), _resolve(item_final), users, pos, neg


def resolve(x):
    """A DeferredFinal's dense table (computed once), any other value as is."""
    return _resolve(x)


class _BprAdamStep(torch.autograd.Function):
    """loss = bpr_loss over one deferred call's batch rows; its backward is the
    whole chain's with the optimizer step in it (bbgr::bpr_adam_backward):
    the weights are updated in place and get no gradient."""

    @staticmethod
    def forward(ctx, u0, i0, users, pos, neg, reg, pending, opt):
        from . import ops
        key, K, maps = pending.step
        mg = opt.masters([u0, i0], maps) if maps is not None else None
        if mg is not None:   # the optimizer's graph-ordered copies are current
            uf, itf = ops.propagate_rows_graph(mg[0], mg[1], users, torch.cat([pos, neg]),
                                               key, K)
        else:
            uf, itf = pending.rows_fn(users, torch.cat([pos, neg]))
        loss = ops.bpr_loss(uf, itf, u0, i0, users, pos, neg, float(reg), None, 0.0)
        ctx.save_for_backward(uf, itf, u0, i0, users, pos, neg)
        ctx.reg, ctx.chain, ctx.opt = float(reg), pending.step, opt
        return loss

    @staticmethod
    def backward(ctx, g):
        from . import ops
        uf, itf, u0, i0, users, pos, neg = ctx.saved_tensors
        key, K, maps = ctx.chain

        def run(states, group, corr):
            su, si = states
            b1, b2 = group["betas"]
            # input-order pair: the Adam updates the graph-ordered master copies
            # (built now if missing or stale) and writes the caller's rows
            mg = ctx.opt.masters([u0, i0], maps, create=True) if maps is not None else None
            ops.bpr_adam_backward(g.detach(), uf, itf, u0.detach(), i0.detach(), users, pos,
                                  neg, ctx.reg, key, K, su["exp_avg"], su["exp_avg_sq"],
                                  si["exp_avg"], si["exp_avg_sq"], float(group["lr"]),
                                  float(b1), float(b2), float(group["eps"]),
                                  float(group["weight_decay"]), corr[0][0], corr[0][1],
                                  corr[1][0], corr[1][1], maps is not None,
                                  None if mg is None else mg[0], None if mg is None else mg[1])
            run.masters_updated = mg is not None

        # an input-order pair: the moments live in the graph's row order
        # (FusedAdam converts them once, and back at its state_dict boundary)
        ctx.opt.step_in_backward([u0, i0], run, row_maps=maps)
        return (None,) * 8


def fused_bpr_step(user_final, item_final, users, pos, neg, reg_weight: float):
    """bpr_loss of one deferred propagate() call with bbgr.optim.FusedAdam(
    fuse_backward=True) owning both weights (GS, num_layers >= 2, eager): the
    loss, whose backward runs the optimizer step (optim.FusedAdam). None when
    that does not apply (the caller takes the usual path)."""
    if not (isinstance(user_final, DeferredFinal) and isinstance(item_final, DeferredFinal)):
        return None
    p = user_final._pending
    if (item_final._pending is not p or user_final._side != 0 or item_final._side != 1
            or p.out is not None or p.step is None or p.step[1] < 2 or not p.grad
            or not torch.is_grad_enabled()):
        return None
    u0, i0 = p.u0, p.i0
    if not (u0.requires_grad and i0.requires_grad and u0.is_leaf and i0.is_leaf
            and u0.is_contiguous() and i0.is_contiguous()):
        return None
    from .optim import backward_optimizer
    opt = backward_optimizer(u0, i0)
    if opt is None:
        return None
    p._check()
    dev = u0.device
    users, pos, neg = (torch.as_tensor(t).to(device=dev, dtype=torch.int64).contiguous()
                       for t in (users, pos, neg))
    return _BprAdamStep.apply(u0, i0, users, pos, neg, float(reg_weight), p, opt)
