"""User-row sharded training over torch.distributed (RCCL on MI355X).

SURVEY §8(e). The reference is single-device; this is the build's scale-out:

  * users are cut into `world` contiguous, edge-balanced ranges; rank g owns
    its users' rows, ALL their edges (user-row CSR slice + the item-row CSR
    restricted to those users), their embedding rows and Adam state.
    Item tables and item Adam state are replicated.
  * per layer and direction one exchange: each rank's item-row SpMM writes raw
    partial row sums over ITS users, an in-place all-reduce (sum) completes
    them, then the fused epilogue (layer mean, next-layer feed scale, backward
    addend) runs on the full sums. User-row SpMMs are purely local.
  * BPR: each rank samples batch/world of its own users; item gradient
    contributions are all-reduced once per step; the ego-L2 item term is
    applied from the all-gathered (pos, neg) indices on every rank (identical
    values, so replicas stay bitwise identical). The loss is the mean over ranks.

Item degrees (and therefore every item scale) are global: the per-rank item
degree counts are all-reduced at setup.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from ._lib import OP_SYM, call, ld, ptr, stream_handle
from .bpr import bpr_args
from .graph import BipartiteGraph, Scales
from .optim import adam_step
from .propagate import OperatorPair, backward, forward
from .sampler import PopMixSampler, nonempty_rows, shuffle
from .trainer import VARIANTS


def partition_users(deg_u: np.ndarray, world: int) -> np.ndarray:
    """Contiguous user ranges with ~equal edge counts: bounds[world+1]."""
    deg_u = np.asarray(deg_u, np.int64)
    U = deg_u.size
    csum = np.concatenate([[0], np.cumsum(deg_u)])
    E = int(csum[-1])
    bounds = np.searchsorted(csum, [E * g // world for g in range(world + 1)], side="left")
    bounds[0], bounds[-1] = 0, U
    return np.maximum.accumulate(bounds).astype(np.int64)


def shard_edges(edges: np.ndarray, lo: int, hi: int) -> np.ndarray:
    """Edges of users [lo, hi) with user ids made local (u - lo)."""
    m = (edges[0] >= lo) & (edges[0] < hi)
    out = edges[:, m].astype(np.int32, copy=True)
    out[0] -= lo
    return out


def global_item_indptr(local_item_degrees: torch.Tensor, group=None) -> torch.Tensor:
    """All-reduce per-rank item degree counts -> global int32 indptr [I+1]."""
    deg = local_item_degrees.to(torch.int64).clone()
    dist.all_reduce(deg, op=dist.ReduceOp.SUM, group=group)
    indptr = torch.zeros(deg.numel() + 1, dtype=torch.int64, device=deg.device)
    indptr[1:] = torch.cumsum(deg, 0)
    return indptr.to(torch.int32)


class ShardedTrainer:
    def __init__(self, edges: np.ndarray, num_users: int, num_items: int,
                 variant: str = "v2_pop", cred=None, emb_dim: int = 64, num_layers: int = 3,
                 lr: float = 1e-3, reg: float = 1e-4, batch_size: int = 8192,
                 neg_mix_pop: float | None = None, neg_pop_gamma: float = 0.75,
                 neg_max_tries: int = 50, lambda_fair: float = 0.0, seed: int = 42,
                 device=None, group=None, u0=None, i0=None):
        _lib.require_gpu()
        if variant not in VARIANTS:
            raise ValueError(f"unknown variant {variant!r}")
        kind, order, mix_default = VARIANTS[variant]
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        dev = torch.device(device) if device is not None else torch.device("cuda")
        self.device = dev
        self.U, self.I, self.d, self.K = num_users, num_items, emb_dim, num_layers
        self.order, self.lr, self.reg = order, lr, reg
        self.lambda_fair = lambda_fair
        self.B_local = max(1, batch_size // self.world)
        self.B_global = self.B_local * self.world

        deg_u = np.bincount(edges[0].astype(np.int64), minlength=num_users)
        self.bounds = partition_users(deg_u, self.world)
        lo, hi = int(self.bounds[self.rank]), int(self.bounds[self.rank + 1])
        self.lo, self.hi, self.U_local = lo, hi, hi - lo
        local = shard_edges(edges, lo, hi)
        self.graph = BipartiteGraph(local, self.U_local, num_items, dev)
        # global item degrees -> scales
        indptr_i = global_item_indptr(self.graph.item_csr.degrees(), group)
        cred_t = None
        if cred is not None and kind != OP_SYM:
            cred_t = torch.as_tensor(np.asarray(cred, np.float32)[lo:hi]).to(dev).contiguous()
        self.scales = _scales(kind, self.graph, indptr_i, cred_t)
        self.pair = OperatorPair.factored(self.graph, self.scales)

        f32 = dict(dtype=torch.float32, device=dev)
        if u0 is None:   # the same global init on every rank; keep my rows
            g = torch.Generator(device="cpu").manual_seed(seed)
            au = (6.0 / (num_users + emb_dim)) ** 0.5
            ai = (6.0 / (num_items + emb_dim)) ** 0.5
            u0 = (torch.rand(num_users, emb_dim, generator=g) * 2 - 1) * au
            i0 = (torch.rand(num_items, emb_dim, generator=g) * 2 - 1) * ai
        self.user_w = torch.as_tensor(u0, dtype=torch.float32)[lo:hi].to(dev).contiguous()
        self.item_w = torch.as_tensor(i0, dtype=torch.float32).to(dev).contiguous()
        z = lambda n: torch.zeros(n, emb_dim, **f32)  # noqa: E731
        self.m_u, self.v_u = z(self.U_local), z(self.U_local)
        self.m_i, self.v_i = z(num_items), z(num_items)
        self.uf, self.itf = z(self.U_local), z(num_items)
        self.g_uf, self.g_if = z(self.U_local), z(num_items)
        self.g_u0, self.g_i0 = z(self.U_local), z(num_items)
        self.parts = torch.empty(3 * self.B_local, **f32)
        self.loss = torch.zeros((), **f32)
        self.dloss = torch.full((), 1.0 / self.world, **f32)   # mean over the global batch
        self.ws: dict = {}
        self.pop = None
        if lambda_fair != 0.0:
            di = self.scales.deg_i
            self.pop = (di / di.max().clamp(min=1.0)).contiguous()
        mix = mix_default if neg_mix_pop is None else neg_mix_pop
        self.sampler = PopMixSampler(self.graph.user_csr, None if mix <= 0 else _GlobalItemCsr(
            indptr_i), num_items, mix_pop=mix, gamma=neg_pop_gamma if mix > 0 else None,
            max_tries=neg_max_tries, seed=seed + 7919 * self.rank)
        self.train_users = nonempty_rows(self.graph.user_csr)
        if self.train_users.numel() == 0:
            raise RuntimeError(f"rank {self.rank}: no train users in its shard")
        self.seed, self.epoch, self.cursor, self.step_count = seed, 0, 0, 0
        self.perm = None
        self.pos = torch.empty(self.B_local, dtype=torch.int64, device=dev)
        self.neg = torch.empty(self.B_local, dtype=torch.int64, device=dev)
        self.all_items = torch.empty(2 * self.B_global, dtype=torch.int64, device=dev)

    # -- collectives ---------------------------------------------------------
    def _allreduce(self, t: torch.Tensor) -> None:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def next_users(self) -> torch.Tensor:
        n = self.train_users.numel()
        if self.perm is None or self.cursor >= n:
            self.epoch += 1
            self.perm = shuffle(self.train_users, self.seed + 7919 * self.rank, self.epoch)
            self.cursor = 0
        users = self.perm[self.cursor: self.cursor + self.B_local]
        self.cursor += self.B_local
        if users.numel() < self.B_local:   # wrap so every rank keeps a full slice
            self.cursor = n
            users = torch.cat([users, self.perm[: self.B_local - users.numel()]])
        return users

    def step(self) -> torch.Tensor:
        users = self.next_users()
        B = users.numel()
        pos, neg = self.sampler.sample(users, self.pos[:B], self.neg[:B])
        st = stream_handle()
        forward(self.pair, self.user_w, self.item_w, self.K, self.order, out_u=self.uf,
                out_i=self.itf, ws=self.ws, reduce=self._allreduce)
        a = bpr_args(users, pos, neg, self.uf, self.itf, self.user_w, self.item_w, self.reg,
                     self.pop, self.lambda_fair, parts=self.parts[: 3 * B], dloss=self.dloss,
                     g_uf=self.g_uf, g_if=self.g_if)
        call("bbgr_bpr", ctypes.byref(a), st)
        call("bbgr_bpr_reduce", B, ptr(self.parts), float(self.reg), float(self.lambda_fair),
             ptr(self.loss), st)
        self._allreduce(self.g_if)                       # item grads of the global batch
        _all_gather(self.all_items, torch.cat([pos, neg]), self.group)
        backward(self.pair, self.g_uf, self.g_if, self.K, self.order, out_u=self.g_u0,
                 out_i=self.g_i0, ws=self.ws, reduce=self._allreduce)
        alpha = 2.0 * self.reg / self.B_global            # ego L2 (Version-2:503-507)
        call("bbgr_rows_axpy", B, ptr(users), alpha, ptr(self.user_w), ld(self.user_w),
             ptr(self.g_u0), ld(self.g_u0), self.d, st)
        call("bbgr_rows_axpy", self.all_items.numel(), ptr(self.all_items), alpha,
             ptr(self.item_w), ld(self.item_w), ptr(self.g_i0), ld(self.g_i0), self.d, st)
        self.step_count += 1
        adam_step(self.user_w, self.g_u0, self.m_u, self.v_u, self.step_count, self.lr)
        adam_step(self.item_w, self.g_i0, self.m_i, self.v_i, self.step_count, self.lr)
        call("bbgr_rows_zero", B, ptr(users), ptr(self.g_uf), ld(self.g_uf), self.d, st)
        call("bbgr_rows_zero", self.all_items.numel(), ptr(self.all_items), ptr(self.g_if),
             ld(self.g_if), self.d, st)
        self._allreduce(self.loss)
        self.loss.mul_(1.0 / self.world)
        return self.loss


def _all_gather(out: torch.Tensor, inp: torch.Tensor, group) -> None:
    """all_gather_into_tensor (RCCL); list form where the backend lacks it (gloo)."""
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, inp, group=group)
        return
    parts = list(out.chunk(dist.get_world_size(group)))
    dist.all_gather(parts, inp, group=group)
    out.copy_(torch.cat(parts))


class _GlobalItemCsr:
    """Just the item indptr (global degrees) the pop CDF needs."""

    def __init__(self, indptr: torch.Tensor):
        self.indptr = indptr


def _scales(kind: int, graph: BipartiteGraph, indptr_i: torch.Tensor,
            cred: torch.Tensor | None) -> Scales:
    U, I, dev = graph.num_users, graph.num_items, graph.device
    f = lambda n: torch.empty(max(n, 1), dtype=torch.float32, device=dev)  # noqa: E731
    deg_u, deg_i = f(U), f(I)
    p, q, s, t, pt, qs = f(I), f(U), f(U), f(I), f(I), f(U)
    call("bbgr_operator_scales", kind, U, I, ptr(graph.user_csr.indptr), ptr(indptr_i),
         ptr(cred), ptr(deg_u), ptr(deg_i), ptr(p), ptr(q), ptr(s), ptr(t), ptr(pt), ptr(qs),
         stream_handle())
    sc = Scales(kind, p[:I], q[:U], s[:U], t[:I], pt[:I], qs[:U], deg_u[:U], deg_i[:I])
    sc._keep = (indptr_i, cred)
    return sc
