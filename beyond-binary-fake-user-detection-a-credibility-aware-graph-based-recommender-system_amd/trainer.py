"""Fused native training step of the reference's training loop.

One step == Version-2/lighgcn_cu_pop.py:826-866 for one batch of users:
  batch users (epoch permutation, :821-827) -> positive + pop-mix negative
  sampling (:835-849) -> propagate() (:858, 2K SpMMs) -> bpr_loss (:859)
  -> backward (:862, 2K transposed SpMMs) -> Adam (:863).
Everything runs on the device on ONE stream with no host synchronisation;
`loss` stays a device scalar until the caller reads it (the reference reads
it every step with float(loss.item()), :865).

Gradient tables that are sparse by construction (dL/d u_final, dL/d i_final:
only batch rows) are kept all-zero between steps: the BPR kernel scatter-adds
into them and the step re-zeroes exactly the touched rows afterwards.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib
from ._lib import OP_GS, OP_J, OP_METHOD_A, OP_SYM, call, ld, ptr, stream_handle
from .bpr import bpr_args
from .graph import BipartiteGraph
from .optim import AdamRows, DeviceStepState, adam_step
from .propagate import ORDER_GS, ORDER_J, ListLength, OperatorPair, backward, forward
from .sampler import PopMixSampler, nonempty_rows, shuffle
from .scatter import RowScatter

VARIANTS = {
    # name: (operator kind, layer order, default negative sampler mix)
    "v2_pop": (OP_GS, ORDER_GS, 0.7),        # Version-2/lighgcn_cu_pop.py
    "cu_message": (OP_GS, ORDER_GS, 0.0),    # version_1/lightgcn_cu_message.py
    "method_a": (OP_METHOD_A, ORDER_GS, 0.0),  # version_1/..._long_tail_exposure.py
    "cu_fair": (OP_J, ORDER_J, 0.0),         # lightgcn_cu.py
    "plain": (OP_SYM, ORDER_J, 0.0),         # lightgcn.py
}

# frontier="auto": masks pay only on graphs whose full-CSR products take well
# over the mask build (~0.05 ms of small launches). Round 6, graph-replayed
# steps: C2 (1M edges) 0.577 ms masked against 0.597 dense, C1 (100K) 0.387
# against 0.300 (profiles/round6/r6c_c{1,2}_frontier_*.json; round 1 measured C2
# the other way, 1.092 vs 1.058 ms, before the products got faster); C4 (50M)
# 16.3 against 22.4. Below this many edges the step runs dense.
FRONTIER_MIN_EDGES = 500_000


def resolve_frontier(frontier, nnz: int) -> bool:
    """`frontier` as given, or the size rule for "auto"."""
    if isinstance(frontier, str):
        if frontier != "auto":
            raise ValueError(f"frontier must be True, False or 'auto', got {frontier!r}")
        return nnz >= FRONTIER_MIN_EDGES
    return bool(frontier)


class FusedTrainer:
    def __init__(self, graph: BipartiteGraph, variant: str = "v2_pop", cred=None,
                 emb_dim: int = 64, num_layers: int = 3, lr: float = 1e-3,
                 reg: float = 1e-4, batch_size: int = 4096, neg_mix_pop: float | None = None,
                 neg_pop_gamma: float = 0.75, neg_max_tries: int = 50,
                 lambda_fair: float = 0.0, seed: int = 42, u0=None, i0=None,
                 frontier="auto", fuse_adam: bool = True):
        _lib.require_gpu()
        if variant not in VARIANTS:
            raise ValueError(f"unknown variant {variant!r}; one of {sorted(VARIANTS)}")
        kind, order, mix_default = VARIANTS[variant]
        self.graph, self.variant, self.order = graph, variant, order
        self.U, self.I, self.d, self.K = graph.num_users, graph.num_items, emb_dim, num_layers
        self.lr, self.reg, self.B = lr, reg, batch_size
        self.lambda_fair, self.seed = lambda_fair, seed
        dev = graph.device
        self.device = dev
        cred_t = None
        if cred is not None and kind != OP_SYM:
            cred_t = torch.as_tensor(np.asarray(cred, np.float32)).to(dev).contiguous()
            cred_t = _internal_rows(graph.user_order, cred_t)
        self.scales = graph.scales(kind, cred_t)
        self.pair = OperatorPair.factored(graph, self.scales)

        f32 = dict(dtype=torch.float32, device=dev)
        if u0 is None:
            g = torch.Generator(device="cpu").manual_seed(seed)
            au = (6.0 / (self.U + emb_dim)) ** 0.5
            ai = (6.0 / (self.I + emb_dim)) ** 0.5
            u0 = (torch.rand(self.U, emb_dim, generator=g) * 2 - 1) * au
            i0 = (torch.rand(self.I, emb_dim, generator=g) * 2 - 1) * ai
        self.user_w = torch.as_tensor(u0, dtype=torch.float32).to(dev).contiguous()
        self.item_w = torch.as_tensor(i0, dtype=torch.float32).to(dev).contiguous()
        if self.user_w.shape != (self.U, emb_dim) or self.item_w.shape != (self.I, emb_dim):
            raise ValueError("initial tables have the wrong shape")
        # tables are given (and generated) by input id; held in the graph's order
        self.user_w = _internal_rows(graph.user_order, self.user_w)
        self.item_w = _internal_rows(graph.item_order, self.item_w)
        z = lambda n: torch.zeros(n, emb_dim, **f32)  # noqa: E731
        self.m_u, self.v_u, self.m_i, self.v_i = z(self.U), z(self.U), z(self.I), z(self.I)
        self.uf = torch.empty(self.U, emb_dim, **f32)
        self.itf = torch.empty(self.I, emb_dim, **f32)
        self.g_uf, self.g_if = z(self.U), z(self.I)         # all-zero between steps
        self.g_u0 = torch.empty(self.U, emb_dim, **f32)
        self.g_i0 = torch.empty(self.I, emb_dim, **f32)
        self.parts = torch.empty(3 * batch_size, **f32)
        self.loss = torch.zeros((), **f32)
        self.ws: dict = {}
        self.pop = None
        if lambda_fair != 0.0:   # lightgcn_cu.py:583-584: pop = deg_i / max(deg_i)
            di = self.scales.deg_i
            self.pop = (di / di.max().clamp(min=1.0)).contiguous()
        mix = mix_default if neg_mix_pop is None else neg_mix_pop
        self.sampler = PopMixSampler(graph.user_csr, graph.item_csr, self.I, mix_pop=mix,
                                     gamma=neg_pop_gamma if mix > 0 else None,
                                     max_tries=neg_max_tries, seed=seed)
        self.train_users = nonempty_rows(graph.user_csr)
        if self.train_users.numel() == 0:
            raise RuntimeError("No train users with interactions. Check your threshold/split.")
        self.epoch, self.cursor, self.step_count = 0, 0, 0
        self.perm = None
        # pos and neg of a batch of B live in posneg[:B] / posneg[B:2B], so the
        # item-gradient scatter takes one contiguous index vector
        self.posneg = torch.empty(2 * batch_size, dtype=torch.int64, device=dev)
        self.pos, self.neg = self.posneg[:batch_size], self.posneg[batch_size:]
        # deterministic BPR gradient: per-triple rows, then a fixed-order scatter
        self.contrib = torch.empty(3 * batch_size, emb_dim, **f32)
        self.scatter = RowScatter()
        # Exact frontier sparsity: a step reads the final tables only at batch
        # rows, and its loss gradient is non-zero only there. Masks (1 byte per
        # node) restrict the last forward layer to the rows it feeds and let the
        # first backward products skip exact-zero source rows. Loss, gradients
        # and updates are bitwise identical to the dense step (tested).
        self.frontier = resolve_frontier(frontier, graph.item_csr.nnz)
        self.mask_u = _lib.byte_mask(self.U, dev)
        # (whole 4-byte words: bbgr_mark_list sets the item bytes by word atomics)
        self.mask_i = _lib.byte_mask(self.I, dev)
        # The first backward item product reads only the batch users' rows of
        # gU (81k of 50M edges at C4) but would scan every index of its
        # frontier rows (20.6M) to find them: a bitmap over the item-CSR slots
        # of the batch users' edges (set with the masks, cleared after the
        # step) lets it test 64 edges per load (bbgr_spmm_args.src_bits;
        # bitwise the mask's result). Full-width tables only (narrow column
        # shards keep the mask).
        self.slot_map = self.slot_bits = None
        if self.frontier and emb_dim >= 64:
            self.slot_map = graph.user_item_slots()
            self.slot_bits = torch.zeros(graph.item_csr.nnz // 32 + 4, dtype=torch.int32,
                                         device=dev)
        # GS: the item frontier also as a row list, built by the marking itself
        # (bbgr_mark_list; length on the device, so a captured step keeps it):
        # the first backward item product then visits the frontier's rows
        # (63k at C4) instead of testing the mask byte of every item row.
        # Its launches take the list at its length (P.ListLength) when the step
        # runs eagerly, at its capacity with the device count when captured.
        # BBGR_TAGGED=1 (GS, K >= 2, a two-row user CSR): the first forward user
        # product writes the user CSR's column indices tagged with the item
        # frontier (bit 31 = dead item, bbgr_spmm_args.tag_out), and the first
        # backward user product reads the frontier from them instead of loading
        # the mask byte of every edge (src_tagged; bitwise the mask launch).
        # Off by default: at C4 the reader drops 0.905 -> 0.770 ms but the
        # writer's 50M extra mask-byte loads cost the forward product +0.26 ms
        # (1.467 -> 1.723 ms; profiles/round6/r6e_tagged_ab.txt).
        self.tagged = None
        uc = graph.user_csr
        if (self.frontier and order == ORDER_GS and num_layers >= 2 and emb_dim >= 64
                and uc.nnz <= 24 * uc.n_rows and os.environ.get("BBGR_TAGGED", "0") == "1"):
            self.tagged = torch.empty(max(uc.nnz, 1), dtype=torch.int32, device=dev)
        # Frontier: the item mask also packed one bit per item after the
        # marking (bbgr_mask_pack) for the first backward user product's
        # per-edge test (bbgr_spmm_args.src_mask_bits; bitwise the byte test;
        # BBGR_MASK_BITS=0 keeps the bytes for A/B)
        self.mask_i_bits = None
        if (self.frontier and num_layers >= 1
                and os.environ.get("BBGR_MASK_BITS", "1") != "0"):
            self.mask_i_bits = torch.zeros(self.I // 32 + 1, dtype=torch.int32, device=dev)
        self.item_list = self.item_count = self.item_len = None
        # GS frontier: the step's bookkeeping (masks, list, slot bits, and the
        # sparse gradient rows' reset) runs as one launch at each end of the
        # step (bbgr_batch_begin / bbgr_batch_end) instead of ~11 small ones;
        # same bytes set and restored (BBGR_BATCH_FUSED=0 keeps the separate
        # launches for A/B).
        self.batch_fused = (self.frontier and order == ORDER_GS
                            and os.environ.get("BBGR_BATCH_FUSED", "1") != "0")
        self._fused_pending = False
        if self.frontier and order == ORDER_GS:
            self.item_list = torch.empty(max(self.I, 1), dtype=torch.int64, device=dev)
            self.item_count = torch.zeros(1, dtype=torch.int64, device=dev)
            # a host wait for the list's length is free only behind the dense
            # forward layers (K >= 2); at K = 1 its consumer is the next launch
            self.item_len = ListLength(self.item_count, wait=num_layers >= 2)
        # Fused optimizer (GS order): the user Adam runs inside the last backward
        # product's epilogue and the item Adam reads gI/(K+1) straight from the
        # sparse BPR gradient table (grad_scale), so neither weight-gradient
        # table is written or re-read. g_u0 / g_i0 are then not materialised;
        # fuse_adam=False keeps them (the gradient-parity tests read them).
        self.fuse_adam = bool(fuse_adam) and (
            (order == ORDER_GS and num_layers >= 1) or (order == ORDER_J and num_layers >= 2))
        # device-resident step scalars (Adam t, sampler counter) for graph
        # capture; None = host scalars in the kernel arguments (eager default)
        self.dev_state: DeviceStepState | None = None

    def enable_device_state(self, max_steps: int = 1 << 20) -> None:
        """Keep the Adam step and the sampler counter on the device from now on
        (bbgr_step_begin), so a step captured once replays correctly. Results
        are bitwise those of the host-scalar path."""
        if self.dev_state is None:
            self.dev_state = DeviceStepState(self.device, self.step_count, self.sampler.counter,
                                             max_steps)

    # -- batching ---------------------------------------------------------------
    def next_users(self) -> torch.Tensor:
        """The next batch slice of the epoch permutation, as INTERNAL row ids
        (== input ids unless the graph is degree-ordered; step() takes input ids)."""
        n = self.train_users.numel()
        if self.perm is None or self.cursor >= n:
            self.epoch += 1
            self.perm = shuffle(self.train_users, self.seed, self.epoch)
            self.cursor = 0
        users = self.perm[self.cursor: self.cursor + self.B]
        self.cursor += self.B
        return users

    # -- one step ----------------------------------------------------------------
    def step(self, users: torch.Tensor | None = None) -> torch.Tensor:
        """One training step over `users` (input ids; default: the next slice of
        the epoch permutation)."""
        listed = users is None   # epoch-permutation slices never repeat a user
        if users is None:
            users = self.next_users()
        else:
            users = users.to(device=self.device, dtype=torch.int64)
            if self.graph.user_order is not None:
                users = self.graph.user_order.to_internal(users)
            users = users.contiguous()
        return self._step(users, listed)

    def _step(self, users: torch.Tensor, listed: bool) -> torch.Tensor:
        """The step on internal user ids (`listed`: no repeated user). Issues
        device work only, so it can be captured (GraphedStep)."""
        if self.dev_state is not None:   # (the kernels clamp t to the exact table)
            self.dev_state.begin()
        self._last_users = users
        B = users.numel()
        self.pos, self.neg = self.posneg[:B], self.posneg[B:2 * B]
        pos, neg = self.sampler.sample(users, self.pos, self.neg,
                                       state=None if self.dev_state is None
                                       else self.dev_state.state)
        st = stream_handle()
        masks = self._set_masks(users, pos, neg, 1) if self.frontier else None
        forward(self.pair, self.user_w, self.item_w, self.K, self.order, out_u=self.uf,
                out_i=self.itf, ws=self.ws,
                final_rows=None if masks is None else
                (masks[0], masks[1], users if listed else None, self._flist(masks)),
                tag=self._tag(masks))
        # (a caller's batch may repeat a user: its last user layer then runs on
        # the de-duplicated mask instead of a row list, whose repeated rows
        # would update the in-place accumulator twice)
        self._bpr(users, pos, neg, B)
        # an epoch slice holds distinct users: their rows are added without the sort
        self.scatter(self.g_uf, users, self.contrib[:B], unique=listed)
        self.scatter(self.g_if, self.posneg[: 2 * B], self.contrib[B: 3 * B])
        call("bbgr_bpr_reduce", B, ptr(self.parts), float(self.reg), float(self.lambda_fair),
             ptr(self.loss), st)
        alpha = 2.0 * self.reg / B
        if self.fuse_adam and self.order == ORDER_J:
            self._backward_fused_j(users, self.posneg[: 2 * B], masks, alpha)
        elif self.fuse_adam:
            self._backward_fused(users, self.posneg[: 2 * B], masks, alpha)
        else:
            backward(self.pair, self.g_uf, self.g_if, self.K, self.order, out_u=self.g_u0,
                     out_i=self.g_i0, ws=self.ws, grad_support=masks,
                     src_bits=self._bits(masks), frontier_list=self._flist(masks),
                     tagged=self._tagged(masks), item_mask_bits=self._mask_bits(masks))
            # ego L2 term goes straight to the weight grads (Version-2:503-507):
            # d/de0 reg*mean(|e0|^2) = 2*reg/B * e0 on every (u, pos, neg) row
            call("bbgr_rows_axpy", B, ptr(users), alpha, ptr(self.user_w), ld(self.user_w),
                 ptr(self.g_u0), ld(self.g_u0), self.d, st)
            call("bbgr_rows_axpy", B, ptr(pos), alpha, ptr(self.item_w), ld(self.item_w),
                 ptr(self.g_i0), ld(self.g_i0), self.d, st)
            call("bbgr_rows_axpy", B, ptr(neg), alpha, ptr(self.item_w), ld(self.item_w),
                 ptr(self.g_i0), ld(self.g_i0), self.d, st)
            self.step_count += 1
            adam_step(self.user_w, self.g_u0, self.m_u, self.v_u, self.step_count, self.lr,
                      dev=self.dev_state)
            adam_step(self.item_w, self.g_i0, self.m_i, self.v_i, self.step_count, self.lr,
                      dev=self.dev_state)
        # restore the all-zero invariant of the sparse gradient tables
        if self._fused_pending:   # (+ the masks, list, bits and item side table)
            self._fused_pending = False
            a = self._batch_args(users, g=True)
            call("bbgr_batch_end", ctypes.byref(a), st)
            self.item_len.invalidate()
            return self.loss
        call("bbgr_rows_zero", B, ptr(users), ptr(self.g_uf), ld(self.g_uf), self.d, st)
        call("bbgr_rows_zero", 2 * B, ptr(self.posneg), ptr(self.g_if), ld(self.g_if), self.d,
             st)   # (pos and neg: posneg[:B], posneg[B:2B])
        if masks is not None:
            self._set_masks(users, pos, neg, 0)
        return self.loss

    def _batch_args(self, users, g: bool = False):
        """bbgr_batch_args over the trainer's own batch (posneg halves)."""
        B = users.numel()
        uc = self.graph.user_csr
        bits = getattr(self, "slot_bits", None)
        side = getattr(self, "_g_item_side", None) if g else None
        a = _lib.BatchArgs()
        a.batch = B
        a.users, a.pos, a.neg = ptr(users), ptr(self.posneg), ptr(self.posneg) + 8 * B
        a.n_users, a.n_items = self.U, self.I
        a.user_indptr, a.user_indices = ptr(uc.indptr), ptr(uc.indices)
        a.mask_u, a.mask_i = ptr(self.mask_u), ptr(self.mask_i)
        a.list, a.count = ptr(self.item_list), ptr(self.item_count)
        if bits is not None:
            a.slot_map, a.slot_bits = ptr(self.slot_map), ptr(bits)
        if g:
            a.g_u, a.ld_gu = ptr(self.g_uf), ld(self.g_uf)
            a.g_i, a.ld_gi = ptr(self.g_if), ld(self.g_if)
            if side is not None:
                a.g_side, a.ld_side = ptr(side), ld(side)
        a.d = self.d
        return a

    def _bpr(self, users, pos, neg, B: int) -> None:
        """Fused BPR forward + per-triple gradient rows (bbgr_bpr, contrib mode)."""
        a = bpr_args(users, pos, neg, self.uf, self.itf, self.user_w, self.item_w, self.reg,
                     self.pop, self.lambda_fair, parts=self.parts[: 3 * B],
                     contrib=self.contrib)
        call("bbgr_bpr", ctypes.byref(a), stream_handle())

    def _backward_fused(self, users, item_rows, masks, alpha: float, reduce=None,
                        item_adam: bool = True) -> None:
        """GS backward with Adam fused (see __init__). The ego-L2 rows enter
        through the sparse tables: grad_u0 = out*T + gl*(gU + alpha/gl*u0[b])
        and grad_i0 = gl*(gI + alpha/gl*i0[pos,neg]) (Version-2:503-507).
        item_rows: the batch's (pos, neg) items — of every rank when sharded,
        where `reduce` is the item exchange and gI already holds the global
        batch's item gradient."""
        st = stream_handle()
        B = users.numel()
        gl = 1.0 / (self.K + 1)
        a_gl = alpha / gl
        self.step_count += 1
        adam_u = AdamRows(self.user_w, self.m_u, self.v_u, self.step_count, self.lr,
                          dev=self.dev_state)

        def before_last():
            call("bbgr_rows_axpy", B, ptr(users), a_gl, ptr(self.user_w), ld(self.user_w),
                 ptr(self.g_uf), ld(self.g_uf), self.d, st)

        # The item Adam rides on the last backward item product (a dense launch
        # over every item row, K >= 2): its gradient gI/(K+1) + ego rows is final
        # before the chain starts, so it is formed in a side table (zero off the
        # batch items, like g_if) that the product's epilogue reads, and the
        # 28 B / parameter pass overlaps the product's gathers. Bitwise the
        # separate _item_adam (same additions, same Adam arithmetic).
        side = item_adam and reduce is None and self.K >= 2
        adam_i = None
        if side:
            ga = self._item_grad_side()   # (a -1 "no negative" row is skipped)
            call("bbgr_rows_copy", item_rows.numel(), ptr(item_rows), ptr(self.g_if),
                 ld(self.g_if), ptr(ga), ld(ga), self.d, st)
            call("bbgr_rows_axpy", item_rows.numel(), ptr(item_rows), a_gl, ptr(self.item_w),
                 ld(self.item_w), ptr(ga), ld(ga), self.d, st)
            adam_i = AdamRows(self.item_w, self.m_i, self.v_i, self.step_count, self.lr,
                              dev=self.dev_state, grad=ga, grad_scale=gl)
        backward(self.pair, self.g_uf, self.g_if, self.K, self.order, out_u=self.g_u0,
                 ws=self.ws, grad_support=masks, grad_i0_dense=False, adam_u=adam_u,
                 src_bits=self._bits(masks), frontier_list=self._flist(masks),
                 before_last=before_last, reduce=reduce, adam_i=adam_i,
                 tagged=self._tagged(masks), item_mask_bits=self._mask_bits(masks))
        if side:   # the side table is all-zero between steps (bbgr_batch_end's rows)
            if not getattr(self, "_fused_pending", False):
                call("bbgr_rows_zero", item_rows.numel(), ptr(item_rows), ptr(ga), ld(ga),
                     self.d, st)
        elif item_adam:
            self._item_adam(item_rows, self.g_if, a_gl, gl)

    def _item_grad_side(self) -> torch.Tensor:
        """The fused item Adam's gradient table [I, d], all-zero between steps."""
        ga = getattr(self, "_g_item_side", None)
        if ga is None:
            ga = self._g_item_side = torch.zeros_like(self.g_if)
        return ga

    def _item_adam(self, item_rows, g, a_gl: float, gl: float) -> None:
        """GS item Adam: grad_i0 = gl * (gI + a_gl * i0[pos, neg]) (Version-2:
        503-507), the ego rows added into the sparse table g first."""
        st = stream_handle()
        # duplicates add the same value, so the atomic order cannot matter
        call("bbgr_rows_axpy", item_rows.numel(), ptr(item_rows), a_gl, ptr(self.item_w),
             ld(self.item_w), ptr(g), ld(g), self.d, st)
        adam_step(self.item_w, g, self.m_i, self.v_i, self.step_count, self.lr,
                  grad_scale=gl, dev=self.dev_state)

    def _backward_fused_j(self, users, item_rows, masks, alpha: float) -> None:
        """Jacobi backward (lightgcn_cu.py / lightgcn.py order) with both Adam
        steps fused into the last products' epilogues; the ego-L2 rows enter
        through the sparse tables just before them, as in _backward_fused."""
        st = stream_handle()
        B = users.numel()
        a_gl = alpha / (1.0 / (self.K + 1))
        self.step_count += 1
        adam_u = AdamRows(self.user_w, self.m_u, self.v_u, self.step_count, self.lr,
                          dev=self.dev_state)
        adam_i = AdamRows(self.item_w, self.m_i, self.v_i, self.step_count, self.lr,
                          dev=self.dev_state)

        def before_last():
            call("bbgr_rows_axpy", B, ptr(users), a_gl, ptr(self.user_w), ld(self.user_w),
                 ptr(self.g_uf), ld(self.g_uf), self.d, st)
            call("bbgr_rows_axpy", item_rows.numel(), ptr(item_rows), a_gl, ptr(self.item_w),
                 ld(self.item_w), ptr(self.g_if), ld(self.g_if), self.d, st)

        backward(self.pair, self.g_uf, self.g_if, self.K, self.order, ws=self.ws,
                 grad_support=masks, adam_u=adam_u, adam_i=adam_i, before_last=before_last,
                 src_bits=self._bits(masks), item_mask_bits=self._mask_bits(masks))

    def _set_masks(self, users, pos, neg, value: int):
        """mask_u = batch users; mask_i = batch items (+ N(batch users) for GS,
        whose last user layer reads the NEW item layer)."""
        st = stream_handle()
        B = users.numel()
        call("bbgr_mark_rows", B, ptr(users), value, ptr(self.mask_u), self.U, st)
        uc = self.graph.user_csr
        lst = getattr(self, "item_list", None)
        # pos and neg are one contiguous vector when they are the trainer's own
        # posneg halves (both marked by one launch)
        pn = (pos.data_ptr() == self.posneg.data_ptr()
              and neg.data_ptr() == self.posneg.data_ptr() + 8 * B)
        items = [(2 * B, ptr(self.posneg))] if pn else [(B, ptr(pos)), (B, ptr(neg))]
        if value and pn and getattr(self, "batch_fused", False) and lst is not None:
            _lib.check_word_padded(self.mask_i, self.I, "item mask")
            a = self._batch_args(users)
            call("bbgr_batch_begin", ctypes.byref(a), st)
            self._pack_item_mask()
            if getattr(self, "item_len", None) is not None:
                self.item_len.publish()
            # (the step's end restores all of it in one bbgr_batch_end; a
            # subclass ending with _set_masks(..., 0) restores it just as well)
            self._fused_pending = type(self)._step is FusedTrainer._step
            return self.mask_u, self.mask_i
        if not value:
            self._fused_pending = False
        if value and lst is not None:   # flag + list the frontier (GS)
            _lib.check_word_padded(self.mask_i, self.I, "item mask")
            li = (ptr(self.mask_i), self.I, ptr(lst), ptr(self.item_count), st)
            for n, p in items:
                call("bbgr_mark_list", n, p, None, None, *li)
            call("bbgr_mark_list", B, ptr(users), ptr(uc.indptr), ptr(uc.indices), *li)
            if getattr(self, "item_len", None) is not None:
                self.item_len.publish()
        else:
            for n, p in items:
                call("bbgr_mark_rows", n, p, value, ptr(self.mask_i), self.I, st)
            if self.order == ORDER_GS:
                call("bbgr_mark_neighbors", B, ptr(users), ptr(uc.indptr), ptr(uc.indices),
                     value, ptr(self.mask_i), st)
            if lst is not None:
                self.item_count.zero_()
                if getattr(self, "item_len", None) is not None:
                    self.item_len.invalidate()
        if value:
            self._pack_item_mask()
        if getattr(self, "slot_bits", None) is not None:   # set / clear the batch's bits
            call("bbgr_mark_slots", B, ptr(users), ptr(uc.indptr), ptr(self.slot_map),
                 ptr(self.slot_bits), value, st)
        return self.mask_u, self.mask_i

    def _pack_item_mask(self) -> None:
        """mask_i_bits = mask_i packed (every word rewritten: nothing to clear)."""
        bits = getattr(self, "mask_i_bits", None)
        if bits is not None:
            call("bbgr_mask_pack", self.I, ptr(self.mask_i), ptr(bits), stream_handle())

    def _mask_bits(self, masks):
        """backward(item_mask_bits=...) when the masks are on."""
        return getattr(self, "mask_i_bits", None) if masks is not None else None

    def _tag(self, masks):
        """forward(tag=...): the tagged user-CSR index copy and the item mask."""
        t = getattr(self, "tagged", None)
        self._tag_fresh = masks is not None and t is not None and self.K >= 2
        return (t, masks[1]) if self._tag_fresh else None

    def _tagged(self, masks):
        """backward(tagged=...): the copy, only if this step's forward wrote it
        (a subclass step that runs its own forward never reads a stale copy)."""
        fresh, self._tag_fresh = getattr(self, "_tag_fresh", False), False
        return self.tagged if (fresh and masks is not None) else None

    def _bits(self, masks):
        """The slot bitmap for backward(src_bits=...) when the masks are on."""
        return getattr(self, "slot_bits", None) if masks is not None else None

    def _flist(self, masks):
        """(item row list, device count) for backward(frontier_list=...)."""
        lst = getattr(self, "item_list", None)
        if masks is None or lst is None:
            return None
        ll = getattr(self, "item_len", None)   # (a subclass may point item_count elsewhere)
        return lst, ll if ll is not None and ll.count is self.item_count else self.item_count

    def forward(self):
        """Final (layer-mean) tables, rows by input id."""
        uf, itf = forward(self.pair, self.user_w, self.item_w, self.K, self.order,
                          out_u=self.uf, out_i=self.itf, ws=self.ws)
        return _input_rows(self.graph.user_order, uf), _input_rows(self.graph.item_order, itf)

    def batch(self):
        """(users, pos, neg) of the last step, as input ids (int64)."""
        B = self._last_users.numel()
        users, pos, neg = self._last_users, self.posneg[:B], self.posneg[B:2 * B]
        go, gi = self.graph.user_order, self.graph.item_order
        if go is not None:
            users = go.to_input(users)
        if gi is not None:
            pos, neg = gi.to_input(pos), gi.to_input(neg)
        return users, pos, neg

    def state_dict(self) -> dict:
        """Reference keys (Version-2:903): user_emb.weight / item_emb.weight
        (rows by input id)."""
        return {"user_emb.weight": _input_rows(self.graph.user_order, self.user_w),
                "item_emb.weight": _input_rows(self.graph.item_order, self.item_w)}


class GraphedStep:
    """FusedTrainer.step captured once into a HIP graph (torch.cuda.CUDAGraph)
    and replayed: one graph launch per step instead of ~40 kernel launches
    (the small-graph path, where launch gaps and per-launch ramps are a
    large share of the step: C2). The trainer keeps its Adam step and sampler
    counter on the device (enable_device_state), the batch users are copied
    into a fixed buffer before each replay, and every replay is bitwise the
    eager step (tested). A short last batch of an epoch runs eagerly.

    Capturing needs the step's workspaces to exist: a trainer that has not
    stepped yet runs its first step eagerly here (a real training step)."""

    def __init__(self, trainer: FusedTrainer):
        self.tr = trainer
        trainer.enable_device_state()
        self.first_loss = None
        if trainer.step_count == 0:
            self.first_loss = trainer.step()
        # capture records launches without running them: the buffer's content
        # at capture time is irrelevant
        self.users = torch.zeros(trainer.B, dtype=torch.int64, device=trainer.device)
        host = (trainer.step_count, trainer.sampler.counter)
        # the graph records the launches of THIS configuration
        self._captured = (trainer.frontier, trainer.fuse_adam, trainer.B)
        trainer.pair.prepare_graph(trainer.d)   # the graph's own split-row workspaces
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            trainer._step(self.users, True)
        # capture recorded the step's launches without running them: undo the
        # host mirrors it advanced
        trainer.step_count, trainer.sampler.counter = host
        torch.cuda.synchronize()

    def step(self) -> torch.Tensor:
        tr = self.tr
        if (tr.frontier, tr.fuse_adam, tr.B) != self._captured:
            raise RuntimeError("GraphedStep: the trainer's frontier / fuse_adam / batch size "
                               "changed since capture; build a new GraphedStep")
        users = tr.next_users()
        if users.numel() != tr.B:       # short tail of an epoch: eager (same device state)
            return tr._step(users, True)
        self.users.copy_(users)
        self.graph.replay()
        tr.step_count += 1
        tr.sampler.counter += 1
        tr._last_users = self.users
        tr.pos, tr.neg = tr.posneg[: tr.B], tr.posneg[tr.B: 2 * tr.B]
        return tr.loss


def _internal_rows(order, t: torch.Tensor) -> torch.Tensor:
    return t if order is None else order.rows_to_internal(t)


def _input_rows(order, t: torch.Tensor) -> torch.Tensor:
    return t if order is None else order.rows_to_input(t)
