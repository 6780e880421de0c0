"""The hot-path kernels as registered torch operators, defined in C++.

`csrc/torch_ops.cpp` (libbbgr_torch.so, built by csrc/Makefile) registers
TORCH_LIBRARY(bbgr): each operator has a HIP kernel that issues libbbgr
launches on torch's current stream, a Meta kernel for torch.compile, and the
forward operators an Autograd kernel whose backward is itself a registered
operator. `LightGCN.propagate()` and `LightGCN.bpr_loss()` of the drop-in
modules (Version-2/lighgcn_cu_pop.py:472-508, lightgcn_cu.py:420-463,
lightgcn.py:318-349) call them, so the drop-in step (:858-863 — propagate,
bpr_loss, backward, Adam) survives torch.compile and CUDA-graph capture, and a
libtorch / TorchScript caller reaches the same operators as torch.ops.bbgr.*:

  bbgr::propagate(u0, i0, pair_key, num_layers, order) -> (u_final, i_final)
  bbgr::propagate_rows(u0, i0, users, items, pair_key, num_layers, order)
                                -> (u_final, i_final) valid at the listed rows only
                                (GS; backward: propagate's)
  bbgr::propagate_rows_graph(u0g, i0g, users, items, pair_key, num_layers)
                                -> propagate_rows (GS) from graph-ordered copies of
                                the weights (no autograd; the in-backward step)
  bbgr::propagate_backward(gU, gI, pair_key, num_layers, order) -> (grad_u0, grad_i0)
  bbgr::propagate_backward_rows(iu, vu, gI, num_users, pair_key, num_layers,
                                order, ii=None, vi=None) -> (grad_u0, grad_i0)
                                (gU given as rows; gI too with ii / vi)
  bbgr::jacobi_layer(u, i, pair_key) -> (new_i, new_u)   (+ _backward)
  bbgr::propagate_sym(x0, pair_key, num_layers) -> x_final   (+ _backward)
  bbgr::bpr_loss(uf, itf, ue, ie, users, pos, neg, reg, pop, lambda_fair) -> loss
  bbgr::bpr_loss_backward(dloss, ...) -> (g_uf, g_if, g_ue, g_ie)
  bbgr::bpr_loss_sparse_ego(..., sparse_uf) -> loss   (eager drop-in step: the
      ego gradients, and with sparse_uf dL/d(u_final), go back as sparse rows)

The sparse operators are not tensors: an OperatorPair is registered once with
the C++ side (`pair_key`: its CSRs, plans, scale vectors, feeds and, for an
input-order pair, the vertex maps — bbgr::_register_pair) and the operators
look it up by key; the registration is dropped when the pair is collected.
This module holds no operator definitions: a missing library raises.
"""
from __future__ import annotations

import itertools
import weakref

import torch

from . import _lib

_loaded = False


def load() -> None:
    """Load libbbgr_torch.so (once); raises if it was not built."""
    global _loaded
    if _loaded:
        return
    path = _lib.PKG_DIR / "lib" / "libbbgr_torch.so"
    if not path.exists():
        raise ImportError(f"libbbgr_torch.so not found at {path}; build it with "
                          "`python -c 'import __graft_entry__ as g; g.build()'`")
    _lib.lib()   # libbbgr.so first (the operators call its C ABI)
    torch.ops.load_library(str(path))
    _loaded = True


load()

propagate = torch.ops.bbgr.propagate
propagate_rows = torch.ops.bbgr.propagate_rows
propagate_backward = torch.ops.bbgr.propagate_backward
propagate_backward_rows = torch.ops.bbgr.propagate_backward_rows
jacobi_layer = torch.ops.bbgr.jacobi_layer
jacobi_layer_backward = torch.ops.bbgr.jacobi_layer_backward
propagate_sym = torch.ops.bbgr.propagate_sym
propagate_sym_backward = torch.ops.bbgr.propagate_sym_backward
bpr_loss = torch.ops.bbgr.bpr_loss
bpr_loss_backward = torch.ops.bbgr.bpr_loss_backward
bpr_loss_sparse_ego = torch.ops.bbgr.bpr_loss_sparse_ego
bpr_adam_backward = torch.ops.bbgr.bpr_adam_backward
propagate_rows_graph = torch.ops.bbgr.propagate_rows_graph

# autograd node name of bbgr::propagate (bpr.py reads the graph)
PROPAGATE_NODE = "torch::autograd::CppNode<bbgr_torch::PropagateFn>"
PROPAGATE_ROWS_NODE = "torch::autograd::CppNode<bbgr_torch::PropagateRowsFn>"

_keys = itertools.count(1)


def counters() -> dict:
    """Backward passes the C++ operators have run: {"rows": propagate's
    sparse-rows backward, "dense": the dense backward ops}."""
    r, d = torch.ops.bbgr._counters()
    return {"rows": r, "dense": d}


def _product_entries(prod, io: bool):
    """(tensors, meta) of one propagate.Product for bbgr::_register_pair."""
    from .graph import HOT_BYTES
    c = prod.csr
    first = None
    if prod.vals is None and prod.in_scale is not None:
        first = prod.first_layer_values()
    in_idx = None
    if io:
        prod.input_struct()
        in_idx = c.__dict__["_input_indices"]
    tensors = [c.indptr, c.indices, c.chunks, c.split, prod.vals, prod.in_scale,
               prod.out_scale, first, in_idx]
    meta = [c.n_rows, c.n_cols, c.nnz, c.long_threshold, c.chunk_edges, c.n_chunks,
            c.n_split, int(bool(c.__dict__.get("cols_by_degree", False))),
            int(bool(c.__dict__.get("rows_by_degree", False))),
            int(c.__dict__.get("hot_bytes", HOT_BYTES))]
    return tensors, meta


def pair_key(pair) -> int:
    """The registry key of an OperatorPair (registered with the C++ operators
    on first use; unregistered when the pair is garbage-collected)."""
    k = getattr(pair, "_op_key", None)
    if k is not None:
        return k
    io = pair.io is not None
    tensors, meta = [], []
    for prod in (pair.fwd_item, pair.fwd_user, pair.bwd_item, pair.bwd_user):
        t, m = _product_entries(prod, io)
        tensors += t
        meta += m
    tensors += [pair.feed_fwd_iu, pair.feed_fwd_ui, pair.feed_bwd_iu, pair.feed_bwd_ui]
    if io:
        tensors += [pair.io.user_map, pair.io.item_map, pair.io.user_rank, pair.io.item_rank]
    else:
        tensors += [None] * 4
    meta += [pair.num_users, pair.num_items]
    k = next(_keys)
    torch.ops.bbgr._register_pair(k, tensors, meta)
    pair._op_key = k
    weakref.finalize(pair, torch.ops.bbgr._unregister_pair, k)
    return k
