"""User-row sharded training over torch.distributed (RCCL on MI355X).

SURVEY §8(e). The reference is single-device; this is the build's scale-out:

  * rank g owns a contiguous range of users: their rows, ALL their edges
    (user-row CSR slice + the item-row CSR restricted to those users), their
    embedding rows and Adam state. Item tables and item Adam state are
    replicated on every rank.
  * per layer and direction ONE exchange: each rank's item-row SpMM writes raw
    partial row sums over ITS users; an in-place all-reduce(SUM) completes them;
    the fused epilogue (layer mean, next-layer feed scale, backward addend)
    then runs on the full sums. User-row SpMMs are purely local.
  * the exchange is pipelined: the item rows are cut into edge-balanced
    ranges; range c's all-reduce (async, RCCL's stream) overlaps range c+1's
    SpMM on the compute stream.
  * BPR: each rank samples its own users; the item gradient of the global
    batch is assembled on every rank from the all-gathered (pos, neg) ids and
    per-triple gradient rows by the same fixed-order scatter (no I*d
    all-reduce); the ego-L2 item term uses the same ids; replicas stay
    bitwise identical; the loss is the mean over ranks.
  * frontier sparsity as on one GPU, with the ITEM masks made global by one
    all-reduce of a byte mask per step (every rank must compute every row any
    rank needs before the exchange); the two frontier item products exchange
    only the frontier rows (compacted), not the whole item table.
  * the user Adam runs fused in the last (purely local) backward product and
    the item Adam reads the sparse item gradient, exactly as on one GPU.
  * item ownership (GS, fused Adam): every rank holds the whole item weight
    table but OWNS an equal contiguous range of item rows (internal order): it
    keeps the Adam moments of those rows only and runs the item Adam on them
    (1/N of the replicated pass). A GS step reads the item weights at the
    global batch items only (the layer-mean start and the ego-L2 term; the
    first item product reads user rows), so after the Adam each rank's rows
    of the NEXT step's batch items (prepared one step ahead) are refreshed
    from their owners: one all-gather of 2*B_global rows, each row copied
    from its owner's slot (bit-exact). sync_items() makes the whole table
    current (eval, state_dict).

Two ways to build the shards:
  ShardedTrainer.from_global_edges(edges, U, I, ...)   strong scaling: one
      graph cut into edge-balanced user ranges (global batch split over ranks)
  ShardedTrainer(local_edges, U_local, I, ...)         weak scaling: each rank
      brings its own user shard (local user ids) over the shared item set
Global item degrees (hence every item scale) come from an all-reduce.
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
from .optim import AdamRows, adam_step
from .propagate import (ORDER_GS, OperatorPair, backward, backward_steps, epilogue, forward,
                        forward_steps, spmm)
from .sampler import PopMixSampler, nonempty_rows, shuffle
from .scatter import RowScatter
from .trainer import VARIANTS, FusedTrainer, _internal_rows, resolve_frontier


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


def _all_gather(out: torch.Tensor, inp: torch.Tensor, group) -> None:
    """all_gather_into_tensor (RCCL); list form where the backend lacks it (gloo)."""
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, inp, group=group)
        return
    parts = list(out.chunk(dist.get_world_size(group)))
    dist.all_gather(parts, inp, group=group)
    out.copy_(torch.cat(parts))


def owner_bounds(num_items: int, world: int) -> list[int]:
    """Item ownership: N equal contiguous row ranges, bounds[world+1]."""
    return [num_items * r // world for r in range(world + 1)]


def refresh_from_owners(table: torch.Tensor, rows: torch.Tensor, bounds: list[int],
                        group=None, gather=None) -> None:
    """table[rows] <- the owning ranks' rows (rank r owns [bounds[r], bounds[r+1])):
    one all-gather of every rank's table[rows], then each row copied from its
    owner's slot (exact copies; duplicate rows write the same value).
    `gather(out, inp)`: the all-gather to use (default: torch.distributed's)."""
    n, d = rows.numel(), table.shape[1]
    world = len(bounds) - 1
    if n == 0 or world == 1:
        return
    # a -1 "no negative" row (the sampler gave up) refreshes row 0 instead: a
    # copy of its owner's current value, harmless, and every rank keeps n rows
    rows = rows.clamp(min=0)
    inner = torch.tensor(bounds[1:-1], dtype=torch.int64, device=rows.device)
    mine = table.index_select(0, rows)
    got = torch.empty(world * n, d, dtype=table.dtype, device=table.device)
    if gather is None:
        _all_gather(got, mine, group)
    else:
        gather(got, mine)
    owner = torch.searchsorted(inner, rows, right=True)
    pick = owner * n + torch.arange(n, device=rows.device)
    table.index_copy_(0, rows, got.index_select(0, pick))


def gather_owned(owned: torch.Tensor, bounds: list[int], group=None) -> torch.Tensor:
    """The whole [bounds[-1], d] table from every rank's owned slice (rank r's
    `owned` holds rows [bounds[r], bounds[r+1]))."""
    world = len(bounds) - 1
    sizes = [bounds[r + 1] - bounds[r] for r in range(world)]
    m, d = max(sizes), owned.shape[1]
    pad = torch.zeros(m, d, dtype=owned.dtype, device=owned.device)
    pad[: owned.shape[0]] = owned
    got = torch.empty(world * m, d, dtype=owned.dtype, device=owned.device)
    _all_gather(got, pad, group)
    return torch.cat([got[r * m: r * m + sizes[r]] for r in range(world)])


_DTYPES = {torch.uint8: 0, torch.int32: 1, torch.int64: 2, torch.float32: 3}
_REDOPS = {"sum": 0, "max": 1, "min": 2}


class RcclItemComm:
    """The item exchange through the C ABI's own RCCL communicator
    (bbgr_comm_init / bbgr_allreduce_items) instead of torch.distributed's
    collective machinery. The unique id travels once over `group`; each
    all-reduce is enqueued on a high-priority comm stream behind the compute
    stream's work so far, and wait() makes the compute stream wait for all of
    them.

    inline=True: every collective runs ON the caller's current stream, in
    issue order (bbgr_allreduce_items / bbgr_comm_allreduce /
    bbgr_comm_allgather): no hop to a comm stream and back (two cross-stream
    waits, ~26 us per exchange on MI355X) where nothing is to overlap the
    collective anyway — one column chain, the exchange not cut in ranges.
    The sharded step then routes ALL its collectives (batch ids, masks, BPR
    rows, item refresh, loss) through this one communicator, so every rank's
    collectives run in one order on one stream."""

    def __init__(self, group=None, device=None, inline: bool = False):
        self.inline = bool(inline)
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        ids = (ctypes.c_uint8 * 128)()
        err = None
        if rank == 0:   # (a failure here travels with the id: no rank waits on it)
            try:
                call("bbgr_comm_unique_id", ids)
            except RuntimeError as ex:
                err = ex
        t = torch.tensor([0 if err is None else 1] + list(ids), dtype=torch.uint8)
        if dist.get_backend(group) == "nccl":
            t = t.to(device)
        src = 0 if group is None else dist.get_global_rank(group, 0)
        dist.broadcast(t, src=src, group=group)
        t = t.cpu().tolist()
        if t[0] != 0:
            raise RuntimeError(f"RcclItemComm: no RCCL unique id on rank 0 ({err})")
        ids = (ctypes.c_uint8 * 128)(*t[1:])
        self.comm = ctypes.c_void_p()
        call("bbgr_comm_init", ctypes.byref(self.comm), world, rank, ids)
        self.stream = torch.cuda.Stream(device=device, priority=-1)
        self.pending = False

    def allreduce_async(self, t: torch.Tensor) -> None:
        if self.inline:
            call("bbgr_allreduce_items", self.comm, ptr(t), t.numel(), stream_handle())
            return
        self.stream.wait_stream(torch.cuda.current_stream(t.device))
        t.record_stream(self.stream)   # the allocator must not reuse t before the sum lands
        call("bbgr_allreduce_items", self.comm, ptr(t), t.numel(), self.stream.cuda_stream)
        self.pending = True

    def wait(self) -> None:
        if self.pending:
            torch.cuda.current_stream(self.stream.device).wait_stream(self.stream)
            self.pending = False

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> None:
        """In-place all-reduce of a contiguous tensor on the current stream."""
        if not t.is_contiguous():
            raise ValueError("all_reduce of a non-contiguous tensor")
        call("bbgr_comm_allreduce", self.comm, ptr(t), t.numel(), _DTYPES[t.dtype], _REDOPS[op],
             stream_handle())

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        """out (world * inp.numel() elements, rank-major) <- every rank's inp."""
        if not (out.is_contiguous() and inp.is_contiguous()) or out.dtype != inp.dtype:
            raise ValueError("all_gather: contiguous tensors of one dtype")
        call("bbgr_comm_allgather", self.comm, ptr(inp), ptr(out), inp.numel(),
             _DTYPES[inp.dtype], stream_handle())

    def close(self) -> None:
        if self.comm:
            call("bbgr_comm_destroy", self.comm)
            self.comm = ctypes.c_void_p()


class ItemExchange:
    """The per-layer exchange of item partial sums (propagate's `reduce` hook).

    Dense products (every item row): the SpMM runs over `parts` edge-balanced
    item-row ranges; each range's partial sums are all-reduced asynchronously
    as soon as they are written, overlapping the next range's SpMM; the
    epilogue runs once all ranges are summed.

    Frontier products (a `row_mask`: the last forward item layer and the first
    backward item product of a training step) need only the step's item
    frontier, a GLOBAL row set identical on every rank (`use_rows`). Only
    those rows are computed (row-list SpMM writing listed row list[j] straight
    to row j of a compact table: y_map = bbgr_list_positions) and all-reduced
    — pipelined over the same row ranges — and the compact epilogue finishes
    them: the payload is |frontier|*d*4 bytes instead of I*d*4."""

    def __init__(self, group=None, parts: int = 4, frontier_parts: int = 2):
        self.group, self.parts = group, max(1, int(parts))
        # frontier products are short (0.2-0.9 ms at C4) and their payload small:
        # each extra part costs a launch ramp + a collective call (~30 us) for
        # little overlap, so they are cut coarser than the dense ones
        self.frontier_parts = max(1, int(frontier_parts))
        self.balance_indptr = None   # global item indptr: identical cuts on every rank
        self._rows = None            # (device list, host offsets, event, positions)
        self._offs = None
        self._compact = None
        self._ranges = None          # (csr, ranges, device boundary rows)
        self._ratios = {}            # acc_scale / y_scale vectors (linear exchange)
        self.rank = dist.get_rank(group)
        self.native: RcclItemComm | None = None   # set: bbgr_allreduce_items instead

    def _allreduce_async(self, t: torch.Tensor, works: list) -> None:
        # a collective reduces numel() elements from the data pointer on: a
        # column view would have the wrong elements summed (gloo does not check)
        if not t.is_contiguous():
            raise ValueError("item exchange: all-reduce of a non-contiguous table")
        if self.native is not None:
            self.native.allreduce_async(t)
        else:
            works.append(dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group,
                                         async_op=True))

    def _wait(self, works: list) -> None:
        for w in works:
            w.wait()
        if self.native is not None:
            self.native.wait()

    def __call__(self, t: torch.Tensor) -> None:
        if not t.is_contiguous():
            raise ValueError("item exchange: all-reduce of a non-contiguous table")
        if self.native is not None and self.native.inline:
            self.native.all_reduce(t)
            return
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def ranges(self, csr):
        """The item CSR's frontier row ranges (global-degree cuts) and their
        boundary rows."""
        if self._ranges is None or self._ranges[0] is not csr:
            rg = csr.row_ranges(self.frontier_parts, self.balance_indptr)
            b = [r[0] for r in rg] + [rg[-1][1]] if rg else [0, 0]
            self._ranges = (csr, rg, torch.tensor(b, dtype=torch.int64, device=csr.device))
        return self._ranges[1], self._ranges[2]

    def list_rows(self, csr, row_list: torch.Tensor, count: torch.Tensor,
                  offs: torch.Tensor, offs_host: torch.Tensor, positions=None):
        """A frontier (rows listed ascending in `row_list`, *count of them:
        bbgr_mask_to_list) split at this exchange's range boundaries on the
        stream: offs[k] = listed rows below boundary k (bbgr_list_offsets),
        copied to the pinned offs_host without blocking. `positions` (int32
        [csr.n_rows]): filled with each listed row's list index
        (bbgr_list_positions), the frontier SpMMs' y_map — they then write
        their rows straight into the compact payload. Returns the rows
        use_rows() takes; the host reads the offsets at the first frontier
        product (one event wait). Every column chain's exchange has the same
        ranges, so one split serves them all."""
        _, bounds = self.ranges(csr)
        n = bounds.numel()
        st = stream_handle()
        call("bbgr_list_offsets", n, ptr(bounds), ptr(row_list), ptr(count), ptr(offs), st)
        if positions is not None:
            call("bbgr_list_positions", csr.n_rows, ptr(row_list), ptr(count), ptr(positions),
                 st)
        host = offs_host[:n]
        host.copy_(offs[:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return (row_list, host, ev, positions)

    def use_rows(self, rows) -> None:
        """The step's frontier (list_rows() of it) for the frontier products."""
        self._rows, self._offs = rows, None

    def clear_rows(self) -> None:
        self._rows, self._offs = None, None

    def rows(self):
        """(row list, [offsets into it at each range boundary], positions or
        None) or None."""
        if self._rows is None:
            return None
        lst, host, ev, positions = self._rows
        if self._offs is None:
            ev.synchronize()
            self._offs = [int(v) for v in host.tolist()]
        return lst, self._offs, positions

    def _compact_buf(self, n: int, d: int, device) -> torch.Tensor:
        c = self._compact
        if c is None or c.shape[0] < n or c.shape[1] != d:
            c = self._compact = torch.empty(max(n, 1), d, dtype=torch.float32, device=device)
        return c[:n]

    def item_product(self, prod, x, first, new, kw) -> None:
        src_mask = kw.pop("src_mask", None)
        row_mask = kw.pop("row_mask", None)
        # the slot bitmap of src_mask's live edges: used by the frontier
        # (row-list) launches, where most listed rows' edges are dead
        src_bits = kw.pop("src_bits", None)
        fr = self.rows() if row_mask is not None else None
        works = []
        if fr is not None:
            lst, offs, positions = fr
            rgs, _ = self.ranges(prod.csr)
            d, n = x.shape[1], offs[-1]
            c = self._compact_buf(n, d, x.device)
            t = None if positions is not None else new("partial", prod.csr.n_rows)
            for k, rg in enumerate(rgs):
                a, b = offs[k], offs[k + 1]
                if b <= a:
                    continue
                part = lst[a:b]
                if positions is not None:   # listed row lst[j] -> row j of c
                    spmm(prod, x, first, y=c, y_map=positions, src_mask=src_mask,
                         row_mask=row_mask, row_list=part, rng=rg, src_bits=src_bits)
                else:
                    spmm(prod, x, first, y=t, src_mask=src_mask, row_mask=row_mask,
                         row_list=part, rng=rg, src_bits=src_bits)
                    call("bbgr_rows_gather", b - a, ptr(part), ptr(t), ld(t), ptr(c[a:b]),
                         ld(c), d, stream_handle())
                self._allreduce_async(c[a:b], works)
            self._wait(works)
            epilogue(c, row_list=lst[:n], n_rows=prod.csr.n_rows, **kw)
            return
        y = kw.get("y")
        # linear form: y itself is all-reduced, so it must be one contiguous
        # block (a column chain's output slice is not: partial sums instead)
        if (row_mask is None and y is not None and y.is_contiguous()
                and not (kw.get("add") is not None and kw.get("acc_out") is not None)):
            self._linear_product(prod, x, first, src_mask, y, kw)
            return
        t = new("partial", prod.csr.n_rows)
        for rg in self._dense_order(prod.csr):
            spmm(prod, x, first, y=t, src_mask=src_mask, row_mask=row_mask, rng=rg)
            self._allreduce_async(t[rg[0]:rg[1]], works)
        self._wait(works)
        epilogue(t, row_mask=row_mask, **kw)

    def _dense_order(self, csr):
        """The dense product's row ranges, last one first. Ranges are cut to
        equal edge counts (equal SpMM time); in degree order their ROW counts
        — the all-reduce payloads — grow towards the cold end (C4: 0.3k ...
        483k of 1M rows). Computing the cold ranges first leaves the small
        hot-item range for last, so the collective that cannot overlap
        anything is the smallest one. Results do not depend on the order."""
        return list(reversed(csr.row_ranges(self.parts, self.balance_indptr)))

    def _linear_product(self, prod, x, first, src_mask, y, kw) -> None:
        """Dense product whose output y = ys*T (+ as*add) is linear in the partial
        sums T: every rank writes its own ys*T_r straight into y (rank 0 also
        the addend), the ranges of y are all-reduced in place, and only the
        layer-mean accumulator (if any) needs a pass afterwards, on its masked
        rows, with T recovered as y / ys. No partial table, no full epilogue
        pass. Equal to the partial-sum exchange up to rounding (ys*sum vs
        sum of ys*T_r)."""
        ys, ys_s = kw.get("y_scale"), kw.get("y_scale_s", 1.0)
        sk = dict(y=y, y_scale=ys, y_scale_s=ys_s)
        if self.rank == 0 and kw.get("add") is not None:
            sk.update(add=kw["add"], add_scale=kw.get("add_scale"),
                      add_scale_s=kw.get("add_scale_s", 1.0), add_mask=kw.get("add_mask"))
        works = []
        for rg in self._dense_order(prod.csr):
            spmm(prod, x, first, src_mask=src_mask, rng=rg, **sk)
            self._allreduce_async(y[rg[0]:rg[1]], works)
        self._wait(works)
        if kw.get("acc_out") is not None:
            ratio, ratio_s = self._acc_ratio(kw.get("acc_scale"), ys, ys_s)
            epilogue(y, acc_in=kw.get("acc_in"), acc_out=kw["acc_out"], acc_scale=ratio,
                     acc_scale_s=kw.get("acc_scale_s", 1.0) * ratio_s,
                     gamma=kw.get("gamma", 1.0), acc_mask=kw.get("acc_mask"),
                     row_mask=kw.get("acc_mask"))

    def _acc_ratio(self, acc_scale, ys, ys_s: float):
        """acc_scale / ys per row (0 where ys == 0: such rows have T == 0)."""
        if ys is None:
            return acc_scale, 1.0 / ys_s
        # keyed on the scale tensors themselves (held by the entry), so a freed
        # vector whose address is reused by a different one never matches
        key = (id(acc_scale), id(ys))
        hit = self._ratios.get(key)
        if hit is not None and hit[0] is acc_scale and hit[1] is ys:
            return hit[2], 1.0 / ys_s
        num = torch.ones_like(ys) if acc_scale is None else acc_scale
        r = torch.where(ys != 0, num / ys, torch.zeros_like(ys)).contiguous()
        self._ratios[key] = (acc_scale, ys, r)
        return r, 1.0 / ys_s


def _item_table_owner(fn):
    """Marks a ShardedTrainer method that may read the item table while rows
    owned by other ranks lag (ShardedTrainer.item_w)."""
    import functools

    @functools.wraps(fn)
    def wrapper(self, *args, **kwargs):
        self.__dict__["_inside"] = self.__dict__.get("_inside", 0) + 1
        try:
            return fn(self, *args, **kwargs)
        finally:
            self.__dict__["_inside"] -= 1
    return wrapper


class ShardedTrainer(FusedTrainer):
    """FusedTrainer's step on one user shard (see the module docstring).

    Per step and rank the exchanges are: one byte all-reduce of the item
    frontier mask; 2(K-1) dense item-row all-reduces (pipelined); two
    frontier-row all-reduces (last forward item layer, first backward item
    product); one all-gather of the batch's (pos, neg) ids and their
    per-triple BPR gradient rows, summed on every rank in the same fixed order
    (bbgr_scatter_add_rows), so the item gradient — and with it the item
    Adam step — is bitwise identical on every rank without an I*d all-reduce;
    one scalar all-reduce of the loss. The user Adam runs fused in the last
    (local) backward product as on one GPU."""

    def __init__(self, local_edges: np.ndarray, num_local_users: int, num_items: int,
                 variant: str = "v2_pop", cred=None, emb_dim: int = 64, num_layers: int = 3,
                 lr: float = 1e-3, reg: float = 1e-4, batch_size: int = 8192,
                 neg_mix_pop: float | None = None, neg_pop_gamma: float = 0.75,
                 neg_max_tries: int = 50, lambda_fair: float = 0.0, seed: int = 42,
                 device=None, group=None, u0=None, i0=None, user_offset: int = 0,
                 frontier="auto", exchange_parts: int = 4, fuse_adam: bool = True,
                 sparse_exchange: bool = True, vertex_order: str = "input",
                 frontier_parts: int = 2, native_comm: bool = False,
                 overlap_item_adam: bool | None = None, column_chains: int = 1,
                 own_items: bool = True):
        """local_edges: int32 [2, E_local] with LOCAL user ids; cred / u0: rows of
        this rank's users; i0: the full (replicated) item table; batch_size:
        users per step on THIS rank. vertex_order="degree": local users by
        local degree, items by GLOBAL degree (identical on every rank).
        column_chains=C > 1: the propagation runs as C independent chains over
        d/C-column slices of the tables, each on its own stream, their issue
        interleaved one exchange at a time (_interleave), so one chain's SpMMs
        overlap the other's item all-reduces. own_items: item rows owned by
        ranks (module docstring; GS fused only)."""
        _lib.require_gpu()
        if variant not in VARIANTS:
            raise ValueError(f"unknown variant {variant!r}")
        kind, order, mix_default = VARIANTS[variant]
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        dev = torch.device(device) if device is not None else torch.device("cuda")
        self.device = dev
        self.variant = variant
        self.U, self.I, self.d, self.K = num_local_users, num_items, emb_dim, num_layers
        self.U_local = num_local_users
        self.lo, self.hi = user_offset, user_offset + num_local_users
        self.order, self.lr, self.reg = order, lr, reg
        self.lambda_fair, self.seed = lambda_fair, seed
        self.exchange = ItemExchange(group, exchange_parts, frontier_parts)
        # native_comm: True / "stream" = the item all-reduces through the C ABI's
        # own RCCL communicator on a comm stream; "inline" = every collective of
        # the step through it, on the compute stream (RcclItemComm)
        if native_comm not in (False, True, "stream", "inline", None):
            raise ValueError("native_comm must be False, True, 'stream' or 'inline'")
        inline = native_comm == "inline"
        if inline and int(column_chains) > 1:
            raise ValueError("native_comm='inline' runs one chain (chains overlap their "
                             "exchanges on a shared comm stream)")
        if native_comm:
            self.exchange.native = RcclItemComm(group, dev, inline=inline)
        self._inline = self.exchange.native if inline else None

        def global_degrees(deg: torch.Tensor) -> torch.Tensor:
            g = deg.to(torch.int64)
            dist.all_reduce(g, op=dist.ReduceOp.SUM, group=group)
            return g.to(torch.int32)

        self.graph = BipartiteGraph(local_edges, num_local_users, num_items, dev,
                                    vertex_order=vertex_order, item_degree_hook=global_degrees)
        indptr_i = global_item_indptr(self.graph.item_csr.degrees(), group)
        self.exchange.balance_indptr = indptr_i
        cred_t = None
        if cred is not None and kind != OP_SYM:
            cred_t = torch.as_tensor(np.asarray(cred, np.float32)).to(dev).contiguous()
            cred_t = _internal_rows(self.graph.user_order, cred_t)
        self.scales = _scales(kind, self.graph, indptr_i, cred_t)
        self.pair = OperatorPair.factored(self.graph, self.scales)
        self.chains = self._build_chains(int(column_chains), emb_dim, group, exchange_parts,
                                         frontier_parts, native_comm, indptr_i, dev)

        f32 = dict(dtype=torch.float32, device=dev)
        if u0 is None:   # rank-local stream for users, shared stream for items
            gu = torch.Generator(device="cpu").manual_seed(seed + 104729 * (self.rank + 1))
            gi = torch.Generator(device="cpu").manual_seed(seed)
            au = (6.0 / (num_local_users * self.world + emb_dim)) ** 0.5
            ai = (6.0 / (num_items + emb_dim)) ** 0.5
            u0 = (torch.rand(num_local_users, emb_dim, generator=gu) * 2 - 1) * au
            i0 = (torch.rand(num_items, emb_dim, generator=gi) * 2 - 1) * ai
        self.user_w = torch.as_tensor(u0, dtype=torch.float32).to(dev).contiguous()
        self.item_w = torch.as_tensor(i0, dtype=torch.float32).to(dev).contiguous()
        if self.user_w.shape != (num_local_users, emb_dim) or self.item_w.shape != (num_items, emb_dim):
            raise ValueError("initial tables have the wrong shape")
        self.user_w = _internal_rows(self.graph.user_order, self.user_w)
        self.item_w = _internal_rows(self.graph.item_order, self.item_w)
        self.train_users = nonempty_rows(self.graph.user_csr)
        if self.train_users.numel() == 0:
            raise RuntimeError(f"rank {self.rank}: no train users in its shard")
        # Every rank takes the same number of users per step (the all-gathers of
        # the batch's item rows need equal shapes), and no batch may hold a user
        # twice (the last forward user product updates acc rows in place from a
        # row list): B_local is capped at the smallest shard's train-user count,
        # as the reference's slice perm[start:start+B] caps a batch at the
        # number of train users (Version-2:826-827).
        n_min = torch.tensor([self.train_users.numel()], dtype=torch.int64,
                             device=dev if dist.get_backend(group) == "nccl" else "cpu")
        dist.all_reduce(n_min, op=dist.ReduceOp.MIN, group=group)
        self.B = self.B_local = max(1, min(int(batch_size), int(n_min.item())))
        self.B_global = self.B_local * self.world
        z = lambda n: torch.zeros(n, emb_dim, **f32)  # noqa: E731
        self.m_u, self.v_u = z(num_local_users), z(num_local_users)
        self.fuse_adam = bool(fuse_adam) and order == ORDER_GS and num_layers >= 1
        # item ownership (module docstring): GS with the fused Adam only (the
        # Jacobi order reads the whole item weight table in its first user
        # product, and the unfused path keeps whole gradient tables)
        self.own_items = self.fuse_adam and bool(own_items)
        self.item_bounds = owner_bounds(num_items, self.world)
        self.ia, self.ib = ((self.item_bounds[self.rank], self.item_bounds[self.rank + 1])
                            if self.own_items else (0, num_items))
        self.m_i, self.v_i = z(self.ib - self.ia), z(self.ib - self.ia)
        self._items_stale = False   # some rows of item_w lag their owner's
        self.uf, self.itf = z(num_local_users), z(num_items)
        self.g_uf, self.g_if = z(num_local_users), z(num_items)   # all-zero between steps
        self.g_u0, self.g_i0 = z(num_local_users), z(num_items)
        B = self.B_local
        self.parts = torch.empty(3 * B, **f32)
        self.contrib = torch.empty(3 * B, emb_dim, **f32)
        self.all_contrib = torch.empty(2 * self.B_global, emb_dim, **f32)
        self.scatter = RowScatter()
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
        self.epoch, self.cursor, self.step_count = 0, 0, 0
        self.perm = None
        # one decision for every rank: the size rule on the GLOBAL edge count
        self.frontier = resolve_frontier(frontier, int(indptr_i[-1]))
        self.dev_state = None   # host step scalars (the sharded step is not graph-captured)
        # GS item Adam on a side stream beside the backward chain: its gradient
        # (gI/(K+1) + ego rows) is final once the all-gathered BPR rows are
        # summed, and with N > 1 the chain waits on its dense exchanges, so the
        # Adam pass (28 B/param over the replicated item table) fills link-bound
        # time instead of following the chain. At N = 1 it only contends with the
        # SpMMs for HBM (measured slower), hence the default.
        if overlap_item_adam is None:
            overlap_item_adam = self.world > 1
        self.overlap_item_adam = bool(overlap_item_adam) and self.fuse_adam
        self.g_adam = z(num_items) if self.overlap_item_adam else None
        self._adam_stream = torch.cuda.Stream(device=dev) if self.overlap_item_adam else None
        # sparse frontier exchange: the step's global item frontier as a row list
        self.sparse_exchange = bool(sparse_exchange) and self.frontier
        # the step's batch and frontier, double-buffered: step t prepares step
        # t+1's (users, negatives, global item mask, frontier row list and its
        # range offsets) before its own forward. Nothing in it depends on the
        # weights, so the values are those of preparing it at t+1; but the
        # host read of the offsets at t+1's first frontier product then finds
        # them copied a step ago instead of waiting for the GPU to get there
        # (at N = 8 that wait serialised host issue and GPU work).
        n_bounds = max(exchange_parts, frontier_parts) + 2
        # the first backward item product's slot bitmap (FusedTrainer): the
        # rank's batch users' edges in its item-CSR order, per front; full-width
        # tables only (column chains run narrow kernels, which keep the mask)
        self.slot_map = None
        if self.frontier and emb_dim >= 64 and not self.chains:
            self.slot_map = self.graph.user_item_slots()
        n_bits = self.graph.item_csr.nnz // 32 + 4 if self.slot_map is not None else 0
        self._fronts = [_Front(B, self.B_global, num_local_users, num_items, n_bounds, dev,
                               n_bits) for _ in range(2)]
        self._next = None
        self._list_ws = None
        self._list_need = None
        self._use(self._fronts[0])

    @classmethod
    def from_global_edges(cls, edges: np.ndarray, num_users: int, num_items: int,
                          variant: str = "v2_pop", cred=None, batch_size: int = 8192,
                          u0=None, i0=None, group=None, seed: int = 42, **kw):
        """Strong scaling: cut ONE graph into edge-balanced user ranges; the
        global batch is split over the ranks."""
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        deg_u = np.bincount(edges[0].astype(np.int64), minlength=num_users)
        bounds = partition_users(deg_u, world)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        emb_dim = kw.get("emb_dim", 64)
        if u0 is None:   # the same global init on every rank; keep my rows
            g = torch.Generator(device="cpu").manual_seed(seed)
            au = (6.0 / (num_users + emb_dim)) ** 0.5
            ai = (6.0 / (num_items + emb_dim)) ** 0.5
            u0 = (torch.rand(num_users, emb_dim, generator=g) * 2 - 1) * au
            i0 = (torch.rand(num_items, emb_dim, generator=g) * 2 - 1) * ai
        u0 = u0[lo:hi]
        c = None if cred is None else np.asarray(cred, np.float32)[lo:hi]
        tr = cls(shard_edges(edges, lo, hi), hi - lo, num_items, variant, cred=c,
                 batch_size=max(1, batch_size // world), u0=u0, i0=i0, group=group,
                 seed=seed, user_offset=lo, **kw)
        tr.bounds = bounds
        return tr

    # -- the item weight table ----------------------------------------------
    @property
    def item_w(self) -> torch.Tensor:
        """The item weight table (internal rows). With item ownership at N > 1
        a step updates only this rank's owned rows and the next batch's item
        rows are refreshed from their owners, so between steps the other rows
        lag the owners' values. Reading it then raises instead of returning
        stale rows: call sync_items() on every rank first (collective), or read
        sync_items()["item_w"]. The reference's weights are always current
        (Version-2/lighgcn_cu_pop.py:863); step(), forward(), state_dict() and
        sync_items() read it internally."""
        if self.__dict__.get("_items_stale") and not self.__dict__.get("_inside", 0):
            raise RuntimeError(
                "ShardedTrainer.item_w: item rows owned by other ranks are stale between "
                "steps (item ownership, N > 1); call sync_items() on every rank first "
                "(collective), or read sync_items()['item_w']")
        return self.__dict__["_item_table"]

    @item_w.setter
    def item_w(self, t: torch.Tensor) -> None:
        self.__dict__["_item_table"] = t

    def _build_chains(self, n: int, emb_dim: int, group, parts: int, frontier_parts: int,
                      native_comm: bool, indptr_i, dev) -> list:
        if n == 1:
            return []
        from .columns import WIDTHS
        if n < 1 or emb_dim % n or emb_dim // n not in WIDTHS:
            raise ValueError(f"cannot run {n} column chains over {emb_dim} columns "
                             f"(slice widths must be one of {WIDTHS})")
        w = emb_dim // n
        chains = []
        for c in range(n):
            # every chain on the ONE group (and one native communicator): the
            # collectives run in issue order on its comm stream on every rank,
            # and the chains' issue is interleaved per exchange (_interleave),
            # so one chain's all-reduce is on the wire while the other computes
            # (two communicators could start their kernels in different orders
            # on different ranks)
            ex = self.exchange if c == 0 else ItemExchange(group, parts, frontier_parts)
            if c > 0:
                ex.balance_indptr = indptr_i
                ex.native = self.exchange.native
            chains.append(_Chain(c * w, (c + 1) * w, ex, torch.cuda.Stream(device=dev), {}))
        # the first-product slot values are built lazily on first use; build
        # them now, on this stream, before two chain streams could race for them
        for prod in (self.pair.fwd_item, self.pair.fwd_user, self.pair.bwd_item,
                     self.pair.bwd_user):
            if prod.vals is None and prod.in_scale is not None:
                prod.first_layer_values()
        return chains

    def _gather(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        """All-gather of the step (batch ids, BPR rows, item refresh)."""
        if self._inline is not None:
            self._inline.all_gather(out, inp)
        else:
            _all_gather(out, inp, self.group)

    def _reduce(self, t: torch.Tensor) -> None:
        """In-place sum over the ranks (item mask bytes, loss)."""
        if self._inline is not None:
            self._inline.all_reduce(t)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def _exchanges(self) -> list:
        return [ch.exchange for ch in self.chains] if self.chains else [self.exchange]

    def close(self) -> None:
        """Destroy the exchange's own RCCL communicator (native_comm), if any;
        collective: every rank calls it before the process group goes."""
        native = self.exchange.native
        if native is not None:
            torch.cuda.synchronize(self.device)
            native.close()
            for ex in self._exchanges():
                ex.native = None

    # -- batching ------------------------------------------------------------
    def next_users(self) -> torch.Tensor:
        n = self.train_users.numel()
        if self.perm is None or self.cursor >= n:
            self.epoch += 1
            self.perm = shuffle(self.train_users, self.seed + 7919 * self.rank, self.epoch)
            self.cursor = 0
        users = self.perm[self.cursor: self.cursor + self.B_local]
        self.cursor += self.B_local
        if users.numel() < self.B_local:   # wrap so every rank keeps a full slice
            # B_local <= n (see __init__): the tail perm[c:n] and the head
            # perm[:B-(n-c)] do not overlap, so the batch has no repeated user
            self.cursor = n
            users = torch.cat([users, self.perm[: self.B_local - users.numel()]])
        return users

    def _use(self, f: "_Front") -> None:
        """Point the step's batch / mask attributes at front f."""
        self.posneg, self.all_items = f.posneg, f.all_items
        B = f.posneg.numel() // 2
        self.pos, self.neg = f.posneg[:B], f.posneg[B:]
        self.mask_u, self.mask_i, self.mask_b = f.mask_u, f.mask_i, f.mask_b
        self.slot_bits = f.slot_bits
        self.item_list, self.item_count = f.item_list, f.item_count

    def _prepare(self, f: "_Front") -> None:
        """One step's batch and frontier into front f, on this stream (and
        the group's): my users and their (pos, neg) items, every rank's (pos,
        neg) ids (all-gather), and with the frontier on, the masks — mask_u:
        my batch users; mask_i: every rank's batch items (+ every rank's
        N(batch users) for GS), made global by a byte all-reduce — and, for
        the sparse exchange, mask_i's rows listed and split at the ranges."""
        users = self.next_users()
        B = users.numel()
        f.users = users
        f.frontier = bool(self.frontier)
        self.sampler.sample(users, f.posneg[:B], f.posneg[B:])
        self._gather(f.all_items, f.posneg)
        f.items_fresh = False
        if not self.frontier:
            return
        st = stream_handle()
        call("bbgr_mark_rows", B, ptr(users), 1, ptr(f.mask_u), self.U, st)
        call("bbgr_mark_rows", 2 * B, ptr(f.posneg), 1, ptr(f.mask_i), self.I, st)
        call("bbgr_mark_rows", f.all_items.numel(), ptr(f.all_items), 1, ptr(f.mask_b),
             self.I, st)
        self._mark_slots(f, 1)
        if self.order == ORDER_GS:
            uc = self.graph.user_csr
            call("bbgr_mark_neighbors", B, ptr(users), ptr(uc.indptr), ptr(uc.indices), 1,
                 ptr(f.mask_i), st)
        self._reduce(f.mask_i)   # byte sum <= world: no wrap
        if self.sparse_exchange:
            self._list_rows(f)

    def _mark_slots(self, f: "_Front", value: int) -> None:
        """Set / clear the slot bits of f's users' edges (bbgr_mark_slots)."""
        if f.slot_bits is not None and f.users is not None:
            uc = self.graph.user_csr
            call("bbgr_mark_slots", f.users.numel(), ptr(f.users), ptr(uc.indptr),
                 ptr(self.slot_map), ptr(f.slot_bits), value, stream_handle())

    def _list_rows(self, f: "_Front") -> None:
        st = stream_handle()
        I = self.I
        if self._list_need is None:   # hipcub's temp size depends on I only
            need = ctypes.c_size_t(0)
            call("bbgr_mask_to_list", I, ptr(f.mask_i), ptr(f.item_list), ptr(f.item_count),
                 None, ctypes.byref(need), st)
            self._list_need = need.value
            self._list_ws = torch.empty(max(need.value, 1), dtype=torch.uint8,
                                        device=self.device)
        have = ctypes.c_size_t(self._list_ws.numel())
        call("bbgr_mask_to_list", I, ptr(f.mask_i), ptr(f.item_list), ptr(f.item_count),
             ptr(self._list_ws), ctypes.byref(have), st)
        f.rows = self.exchange.list_rows(self.graph.item_csr, f.item_list, f.item_count,
                                         f.offs, f.offs_host, f.positions)

    def _item_adam_beside(self) -> torch.cuda.Event:
        """The item Adam of this step on the side stream: its gradient rows are
        copied out of g_if (which the backward chain still reads as its addend)
        into g_adam, the ego rows are added there, Adam runs, and g_adam's rows
        are zeroed again. Values are those of the in-chain Adam bit for bit.
        The step count it uses is the one _backward_fused is about to take."""
        main = torch.cuda.current_stream()
        side = self._adam_stream
        side.wait_stream(main)
        rows = self.all_items
        gl = 1.0 / (self.K + 1)
        a_gl = (2.0 * self.reg / self.B_global) / gl
        step_count, self.step_count = self.step_count, self.step_count + 1
        with torch.cuda.stream(side):   # (a -1 "no negative" row is skipped)
            call("bbgr_rows_copy", rows.numel(), ptr(rows), ptr(self.g_if), ld(self.g_if),
                 ptr(self.g_adam), ld(self.g_adam), self.d, stream_handle())
            self._item_adam(rows, self.g_adam, a_gl, gl)
            call("bbgr_rows_zero", rows.numel(), ptr(rows), ptr(self.g_adam),
                 ld(self.g_adam), self.d, stream_handle())
        self.step_count = step_count
        for t in (rows, self.g_if, self.g_adam, self.item_w, self.m_i, self.v_i):
            t.record_stream(side)
        done = torch.cuda.Event()
        done.record(side)
        return done

    def _item_adam(self, item_rows, g, a_gl: float, gl: float) -> None:
        """GS item Adam (FusedTrainer._item_adam) on this rank's OWNED item rows
        (all rows without item ownership); the rows of the other ranks go stale
        here until refreshed (_refresh_items / sync_items)."""
        if not self.own_items:
            super()._item_adam(item_rows, g, a_gl, gl)
            return
        st = stream_handle()
        call("bbgr_rows_axpy", item_rows.numel(), ptr(item_rows), a_gl, ptr(self.item_w),
             ld(self.item_w), ptr(g), ld(g), self.d, st)
        a, b = self.ia, self.ib
        if b > a:
            adam_step(self.item_w[a:b], g[a:b], self.m_i, self.v_i, self.step_count, self.lr,
                      grad_scale=gl)
        self._items_stale = self.world > 1

    def _refresh_items(self, rows: torch.Tensor) -> None:
        """item_w[rows] <- the owners' current values (refresh_from_owners)."""
        if self._items_stale:
            refresh_from_owners(self.item_w, rows, self.item_bounds, self.group,
                                gather=self._gather)

    @_item_table_owner
    def sync_items(self) -> dict:
        """Collective (every rank calls it): make the whole item weight table
        current on this rank and return the item tables by internal row:
        {"item_w", "m_i", "v_i"} (the Adam moments gathered from their owners).
        Without item ownership the local tables are returned as they are."""
        if not self.own_items or self.world == 1:
            return {"item_w": self.item_w, "m_i": self.m_i, "v_i": self.v_i}
        a, b, g = self.ia, self.ib, self.group
        self.item_w.copy_(gather_owned(self.item_w[a:b].contiguous(), self.item_bounds, g))
        self._items_stale = False
        return {"item_w": self.item_w, "m_i": gather_owned(self.m_i, self.item_bounds, g),
                "v_i": gather_owned(self.v_i, self.item_bounds, g)}

    @_item_table_owner
    def forward(self):
        """Final (layer-mean) tables of the rank's users and of every item,
        rows by input id (collective: the item sums are exchanged)."""
        self.sync_items()
        uf, itf = forward(self.pair, self.user_w, self.item_w, self.K, self.order, out_u=self.uf,
                          out_i=self.itf, ws=self.ws, reduce=self.exchange)
        from .trainer import _input_rows
        return _input_rows(self.graph.user_order, uf), _input_rows(self.graph.item_order, itf)

    @_item_table_owner
    def state_dict(self) -> dict:
        """Reference keys (Version-2:903) of this rank's user rows and every
        item row, by input id (collective)."""
        self.sync_items()
        return super().state_dict()

    def pending(self):
        """The batch already prepared for the next step (users as internal
        ids), or None. With prefetch on, after a step the sampler counter,
        epoch and cursor are one batch ahead of step_count: that batch is
        here, and the next step() trains on it as prepared (a caller that
        changes batch or frontier settings between steps should drop it
        with discard_pending() first)."""
        return None if self._next is None else self._next.users

    def discard_pending(self) -> None:
        """Forget the prepared batch and clear its masks; the next step()
        prepares its own (the sampler and the epoch cursor stay where the
        prepared one left them)."""
        f = self._next
        self._next = None
        if f is None:
            return
        if f.frontier and f.users is not None:   # masks are all-zero between uses
            call("bbgr_mark_rows", f.users.numel(), ptr(f.users), 0, ptr(f.mask_u), self.U,
                 stream_handle())
            call("bbgr_mark_rows", f.all_items.numel(), ptr(f.all_items), 0, ptr(f.mask_b),
                 self.I, stream_handle())
            self._mark_slots(f, 0)
            f.mask_i.zero_()
        f.rows = None

    @_item_table_owner
    def step(self, prefetch: bool = True) -> torch.Tensor:
        """One training step. prefetch=False: do not prepare the next step's
        batch (a caller's last step; no batch is sampled and exchanged that
        no step trains on)."""
        if self._next is not None and self._next.frontier != bool(self.frontier):
            self.discard_pending()   # prepared under the other frontier setting
        f = self._next
        if f is None:   # first step (or after discard_pending): nothing prepared
            f = self._fronts[0]
            self._prepare(f)
        nxt = self._fronts[1] if f is self._fronts[0] else self._fronts[0]
        if prefetch:
            self._prepare(nxt)   # the next step's batch and frontier (see __init__)
            self._next = nxt
        else:
            self._next = None
        self._use(f)
        if not f.items_fresh:   # (prepared now, or the last step had no prefetch)
            self._refresh_items(f.all_items)
            f.items_fresh = True
        users, pos, neg = f.users, self.pos, self.neg
        self._last_users = users
        B = users.numel()
        st = stream_handle()
        masks = (self.mask_u, self.mask_i) if self.frontier else None
        if f.rows is not None:
            for ex in self._exchanges():
                ex.use_rows(f.rows)
        final_rows = None if masks is None else (masks[0], masks[1], users, None,
                                                 self.mask_b)
        if self.chains:
            self._forward_chains(final_rows)
        else:
            forward(self.pair, self.user_w, self.item_w, self.K, self.order, out_u=self.uf,
                    out_i=self.itf, ws=self.ws, reduce=self.exchange, final_rows=final_rows)
        a = bpr_args(users, pos, neg, self.uf, self.itf, self.user_w, self.item_w, self.reg,
                     self.pop, self.lambda_fair, parts=self.parts[: 3 * B], dloss=self.dloss,
                     contrib=self.contrib)
        call("bbgr_bpr", ctypes.byref(a), st)
        call("bbgr_bpr_reduce", B, ptr(self.parts), float(self.reg), float(self.lambda_fair),
             ptr(self.loss), st)
        # (every step's batch holds distinct users: next_users)
        self.scatter(self.g_uf, users, self.contrib[:B], unique=True)
        # item gradient of the global batch: every rank's (pos, neg) rows
        # (gathered with the batch) and their per-triple gradient rows, summed
        # in rank-major order
        self._gather(self.all_contrib, self.contrib[B: 3 * B])
        self.scatter(self.g_if, self.all_items, self.all_contrib)
        alpha = 2.0 * self.reg / self.B_global            # ego L2 (Version-2:503-507)
        if self.chains:
            self._backward_chains(users, masks, alpha)
        elif self.fuse_adam and self.overlap_item_adam:
            done = self._item_adam_beside()
            self._backward_fused(users, self.all_items, masks, alpha, reduce=self.exchange,
                                 item_adam=False)
            torch.cuda.current_stream().wait_event(done)
        elif self.fuse_adam:
            self._backward_fused(users, self.all_items, masks, alpha, reduce=self.exchange)
        else:
            backward(self.pair, self.g_uf, self.g_if, self.K, self.order, out_u=self.g_u0,
                     out_i=self.g_i0, ws=self.ws, reduce=self.exchange, grad_support=masks)
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
        if masks is not None:
            call("bbgr_mark_rows", B, ptr(users), 0, ptr(self.mask_u), self.U, st)
            call("bbgr_mark_rows", self.all_items.numel(), ptr(self.all_items), 0,
                 ptr(self.mask_b), self.I, st)
            self._mark_slots(f, 0)
            self.mask_i.zero_()
        if self._next is not None:   # owners' rows of the next step's batch items
            self._refresh_items(self._next.all_items)
            self._next.items_fresh = True
        f.rows = None
        for ex in self._exchanges():
            ex.clear_rows()
        self._reduce(self.loss)
        self.loss.mul_(1.0 / self.world)
        return self.loss


    # -- column chains -------------------------------------------------------
    def _interleave(self, steps) -> None:
        """steps(chain, cols) -> a forward_steps / backward_steps generator per
        chain, each advanced on its chain's stream (after this stream's work so
        far) one exchange at a time, round robin: chain 0's item product and
        all-reduce, chain 1's, chain 0's next products, ... The host order is
        the same on every rank, so the one comm stream runs the collectives in
        the same order everywhere. This stream then waits for every chain."""
        main = torch.cuda.current_stream()
        active = []
        for ch in self.chains:
            ch.stream.wait_stream(main)
            active.append((ch, steps(ch, slice(ch.c0, ch.c1))))
        while active:
            for item in list(active):
                ch, gen = item
                with torch.cuda.stream(ch.stream):
                    try:
                        next(gen)
                    except StopIteration:
                        active.remove(item)
        for ch in self.chains:
            main.wait_stream(ch.stream)

    def _forward_chains(self, final_rows) -> None:
        self._interleave(lambda ch, cs: forward_steps(
            self.pair, self.user_w[:, cs], self.item_w[:, cs], self.K, self.order,
            out_u=self.uf[:, cs], out_i=self.itf[:, cs], ws=ch.ws, reduce=ch.exchange,
            final_rows=final_rows))

    def _backward_chains(self, users, masks, alpha: float) -> None:
        """The backward of every chain on its column slice, then (on this
        stream) what needs whole rows: the item Adam — or, unfused, the ego-L2
        rows and both Adam steps. Per column the arithmetic is the one-chain
        step's, so results match it bit for bit."""
        B = users.numel()
        gl = 1.0 / (self.K + 1)
        a_gl = alpha / gl
        if not self.fuse_adam:
            self._interleave(lambda ch, cs: backward_steps(
                self.pair, self.g_uf[:, cs], self.g_if[:, cs], self.K, self.order,
                out_u=self.g_u0[:, cs], out_i=self.g_i0[:, cs], ws=ch.ws, reduce=ch.exchange,
                grad_support=masks))
            st = stream_handle()
            call("bbgr_rows_axpy", B, ptr(users), alpha, ptr(self.user_w), ld(self.user_w),
                 ptr(self.g_u0), ld(self.g_u0), self.d, st)
            call("bbgr_rows_axpy", self.all_items.numel(), ptr(self.all_items), alpha,
                 ptr(self.item_w), ld(self.item_w), ptr(self.g_i0), ld(self.g_i0), self.d, st)
            self.step_count += 1
            adam_step(self.user_w, self.g_u0, self.m_u, self.v_u, self.step_count, self.lr)
            adam_step(self.item_w, self.g_i0, self.m_i, self.v_i, self.step_count, self.lr)
            return
        done = self._item_adam_beside() if self.overlap_item_adam else None
        self.step_count += 1

        def steps(ch, cs):
            w = ch.c1 - ch.c0
            adam_u = AdamRows(self.user_w[:, cs], self.m_u[:, cs], self.v_u[:, cs],
                              self.step_count, self.lr)

            def before_last():
                call("bbgr_rows_axpy", B, ptr(users), a_gl, ptr(self.user_w[:, cs]),
                     ld(self.user_w), ptr(self.g_uf[:, cs]), ld(self.g_uf), w, stream_handle())
            return backward_steps(self.pair, self.g_uf[:, cs], self.g_if[:, cs], self.K,
                                  self.order, out_u=self.g_u0[:, cs], ws=ch.ws,
                                  grad_support=masks, grad_i0_dense=False, adam_u=adam_u,
                                  before_last=before_last, reduce=ch.exchange)
        self._interleave(steps)
        if done is not None:
            torch.cuda.current_stream().wait_event(done)
        else:
            self._item_adam(self.all_items, self.g_if, a_gl, gl)


class _Chain:
    """One column chain of a ShardedTrainer: columns [c0, c1) of every table,
    its stream, its item exchange (the trainer's group; its own compaction
    buffers and ratio cache) and its workspaces."""

    def __init__(self, c0: int, c1: int, exchange: ItemExchange, stream, ws: dict):
        self.c0, self.c1, self.exchange, self.stream, self.ws = c0, c1, exchange, stream, ws


class _Front:
    """One step's batch and frontier (ShardedTrainer keeps two: the running
    step's and the next one's). Masks are all-zero between uses."""

    def __init__(self, B: int, B_global: int, U: int, I: int, n_bounds: int, dev,
                 n_bits: int = 0):
        i64 = dict(dtype=torch.int64, device=dev)
        self.users = None
        self.posneg = torch.empty(2 * B, **i64)
        self.all_items = torch.empty(2 * B_global, **i64)
        self.mask_u = _lib.byte_mask(U, dev)
        self.mask_i = _lib.byte_mask(I, dev)
        self.item_list = torch.empty(max(I, 1), **i64)
        self.item_count = torch.zeros(1, **i64)
        self.positions = torch.zeros(max(I, 1), dtype=torch.int32, device=dev)
        self.offs = torch.zeros(n_bounds, **i64)
        self.offs_host = torch.zeros(n_bounds, dtype=torch.int64).pin_memory()
        self.rows = None   # ItemExchange.list_rows() of the frontier
        self.frontier = False   # prepared with the frontier masks set
        # every rank's batch items: the item rows whose final value is read
        # (the item layer-mean accumulator is formed there only)
        self.mask_b = _lib.byte_mask(I, dev)
        self.items_fresh = False   # item_w current at all_items (item ownership)
        # slot bitmap of the batch users' edges (all-zero between uses)
        self.slot_bits = (torch.zeros(n_bits, dtype=torch.int32, device=dev) if n_bits
                          else None)


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
