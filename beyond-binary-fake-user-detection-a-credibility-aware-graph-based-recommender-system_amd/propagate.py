"""K-layer LightGCN propagation on the fused HIP SpMM, forward and backward.

Three layer orders exist in the reference:

  GS  (Gauss-Seidel; Version-2/lighgcn_cu_pop.py:472-490, version_1/*):
        i_k = M_iu u_{k-1};  u_k = M_ui i_k          (uses the NEW item table)
  J   (Jacobi; lightgcn_cu.py:420-448):
        i_k = M_iu u_{k-1};  u_k = M_ui i_{k-1}      (uses the OLD item table)
  SYM (lightgcn.py:318-325): x_k = A_hat x_{k-1} on the N x N symmetric
        operator == J on its two off-diagonal blocks.

Final tables are the layer means (Version-2:488-489), fused into the SpMM
epilogue (acc_out = (acc_in + out_scale*T) * gamma, gamma = 1/(K+1) on the
last layer).

Factored operators (graph.Scales) are applied as diag(out) A diag(in): the
producing SpMM writes its output already multiplied by the NEXT product's
input scale (``feed`` vectors pt / qs), so later SpMMs read plain rows and
stream no per-edge weights. The first product of a chain reads the raw
weight table and applies the input scale per gathered row (weight_mode 2).

Backward (autograd of the reference's torch.sparse.mm chain):
with g = dL/d(final) and g' = g/(K+1),
  GS: Gi_k = gI' + M_ui^T Gu_k ; Gu_{k-1} = gU' + M_iu^T Gi_k ; Gu_K = gU'
      grad_u0 = Gu_0, grad_i0 = gI'
  J : Gu_{k-1} = gU' + M_iu^T Gi_k ; Gi_{k-1} = gI' + M_ui^T Gu_k
      (Gu_K = gU', Gi_K = gI'); grad_u0 = Gu_0, grad_i0 = Gi_0
The transposes are the other CSR with the scale roles swapped.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import torch

from . import _lib
from ._lib import call, ld, ptr, stream_handle
from .graph import BipartiteGraph, Csr, Scales

ORDER_GS = "gs"
ORDER_J = "jacobi"


@dataclass
class Product:
    """One sparse product y = diag(out_scale) A diag(in_scale) x (factored) or
    y = M x with explicit per-edge values (generic)."""
    csr: Csr
    vals: torch.Tensor | None
    in_scale: torch.Tensor | None
    out_scale: torch.Tensor | None
    partial: dict
    first_vals: torch.Tensor | None = None
    col_input_map: torch.Tensor | None = None   # internal column id -> input id (int32)

    def input_struct(self):
        """The CSR with INPUT-id column indices (built once, 4 B/edge, shared by
        the products over the same CSR): a first product of an input-order pair
        gathers the caller's input-order table through it."""
        c = self.csr
        st = c.__dict__.get("_input_struct")
        if st is None:
            idx = c.__dict__.get("_input_indices")   # kept by the graph build
            if idx is None:
                if self.col_input_map is None:
                    raise RuntimeError("product has no input-id column map")
                idx = torch.empty(max(c.nnz, 1), dtype=torch.int32, device=c.device)
                call("bbgr_relabel", c.nnz, ptr(c.indices), ptr(self.col_input_map), ptr(idx),
                     stream_handle())
                c.__dict__["_input_indices"] = idx
            st = c.struct(with_plan=True)
            st.indices = ptr(idx)
            c.__dict__["_input_struct"] = st
        return st

    def first_layer_values(self) -> torch.Tensor:
        """in_scale[col] per CSR slot (built once, 4 B/edge): the first product of
        a chain streams these instead of gathering in_scale[col] at random."""
        if self.first_vals is None:
            c = self.csr
            v = torch.empty(max(c.nnz, 1), dtype=torch.float32, device=c.device)
            call("bbgr_gather_scale", c.nnz, ptr(c.indices), ptr(self.in_scale), ptr(v),
                 stream_handle())
            self.first_vals = v
        return self.first_vals

    def workspace(self, d: int):
        """Split-row partials and arrival counters, one set per (width, stream):
        launches on two streams (column chains) must not share counters. A
        graph capture gets a set of its own, so a replay on any stream never
        races eager launches over shared counters: prepared before
        capture by `prepare_graph` (GraphedStep), else allocated inside the
        capture (its zero fill is then part of the graph, re-run per replay)."""
        if self.csr.n_split == 0:
            return None
        dev = self.csr.device
        if torch.cuda.is_current_stream_capturing():
            key = (d, "graph")
        else:
            key = (d, torch.cuda.current_stream(dev).cuda_stream)
        w = self.partial.get(key)
        if w is None:
            w = self.csr.partial_workspace(d)
            self.partial[key] = w
        return w

    def prepare_graph(self, d: int) -> None:
        """Allocate the captured launches' workspace (call outside capture)."""
        if self.csr.n_split and (d, "graph") not in self.partial:
            self.partial[(d, "graph")] = self.csr.partial_workspace(d)


@dataclass
class InputOrder:
    """Vertex maps of an input-order pair: *_map[internal] = input id,
    *_rank[input id] = internal (int32, graph.VertexOrder perm / rank)."""
    user_map: torch.Tensor
    item_map: torch.Tensor
    user_rank: torch.Tensor
    item_rank: torch.Tensor

    def __post_init__(self):   # int64 copies for torch indexing (built once)
        self.user_map64, self.item_map64 = self.user_map.long(), self.item_map.long()
        self.user_rank64, self.item_rank64 = self.user_rank.long(), self.item_rank.long()


class OperatorPair:
    """The four products of one bipartite operator pair (fwd item<-user,
    fwd user<-item, and their transposes for the backward)."""

    def __init__(self, fwd_item: Product, fwd_user: Product, bwd_item: Product,
                 bwd_user: Product, num_users: int, num_items: int,
                 feed_fwd_iu=None, feed_fwd_ui=None, feed_bwd_iu=None,
                 feed_bwd_ui=None):
        self.fwd_item, self.fwd_user = fwd_item, fwd_user
        self.bwd_item, self.bwd_user = bwd_item, bwd_user
        self.num_users, self.num_items = num_users, num_items
        # feed vectors: output scale of a product x input scale of the next one
        self.feed_fwd_iu, self.feed_fwd_ui = feed_fwd_iu, feed_fwd_ui
        self.feed_bwd_iu, self.feed_bwd_ui = feed_bwd_iu, feed_bwd_ui
        self.io: InputOrder | None = None

    def set_input_order(self, user_order, item_order) -> None:
        """The pair's graph is numbered by descending degree (graph.VertexOrder
        per side) but its callers' tables — u0 / i0, the final tables, the
        gradients — stay in INPUT order: the first products gather through
        input-id column indices and the epilogues place input-order rows
        through row maps (bbgr_spmm_args.y_map / acc_map / add_map). The drop-in
        modules get the hot-prefix / streaming policy of the degree order
        without a permute of any table."""
        self.io = InputOrder(user_order.perm, item_order.perm, user_order.rank,
                             item_order.rank)
        self.fwd_item.col_input_map = self.bwd_item.col_input_map = self.io.user_map
        self.fwd_user.col_input_map = self.bwd_user.col_input_map = self.io.item_map

    def prepare_graph(self, d: int) -> None:
        """Workspaces of a graph capture of this pair's products (width d)."""
        for p in (self.fwd_item, self.fwd_user, self.bwd_item, self.bwd_user):
            p.prepare_graph(d)

    @classmethod
    def factored(cls, graph: BipartiteGraph, sc: Scales) -> "OperatorPair":
        Ai, Au = graph.item_csr, graph.user_csr
        wi, wu = {}, {}
        return cls(
            fwd_item=Product(Ai, None, sc.q, sc.p, wi),
            fwd_user=Product(Au, None, sc.t, sc.s, wu),
            bwd_item=Product(Ai, None, sc.s, sc.t, wi),
            bwd_user=Product(Au, None, sc.p, sc.q, wu),
            num_users=graph.num_users, num_items=graph.num_items,
            feed_fwd_iu=sc.pt, feed_fwd_ui=sc.qs, feed_bwd_iu=sc.pt, feed_bwd_ui=sc.qs)

    @classmethod
    def generic(cls, M_iu_csr: Csr, M_ui_csr: Csr, M_ui_T_csr: Csr, M_iu_T_csr: Csr,
                num_users: int, num_items: int) -> "OperatorPair":
        """Arbitrary per-edge values (e.g. a torch sparse COO handed in)."""
        return cls(
            fwd_item=Product(M_iu_csr, M_iu_csr.values, None, None, {}),
            fwd_user=Product(M_ui_csr, M_ui_csr.values, None, None, {}),
            bwd_item=Product(M_ui_T_csr, M_ui_T_csr.values, None, None, {}),
            bwd_user=Product(M_iu_T_csr, M_iu_T_csr.values, None, None, {}),
            num_users=num_users, num_items=num_items)


class SpmmTimer:
    """Brackets every bbgr_spmm launch (incl. its fix-up) with events on the
    launching stream; used by bench.py inside the timed region. With
    `count=True` it records no events and instead counts, on the device, the
    rows and edges each launch actually processes (bench.py's traversed-edge
    figure; run over extra steps outside the timed region)."""

    def __init__(self, count: bool = False, select=None):
        self.count = count
        # select(kind, prod) -> bool: time only those launches (the others run
        # without events, so the timer adds no gaps around them)
        self.select = select
        # (rows, nnz, d, kind, start_event, end_event, table_rows, n_cols, masks)
        self.records = []
        # (kind, masks, table_rows, n_cols, d, rows_t, visited_t, gathered_t): device counts
        self.counts = []

    def summary(self, kind: str = "full", table_rows: int | None = None):
        """{(rows, nnz, d): (launches, total ms)} over one kind of launch:
        "full" (spmm_kernel), "masked" (frontier masks / row lists,
        spmm_masked_kernel) or "adam" (fused Adam epilogue, spmm_adam_kernel);
        `table_rows` keeps only launches over a CSR with that many rows (the
        item-row CSR: the item<-user products)."""
        torch.cuda.synchronize()
        out = {}
        for rows, nnz, d, m, a, b, tr, _, _ in self.records:
            if m != kind or (table_rows is not None and tr != table_rows):
                continue
            k = (rows, nnz, d)
            n, ms = out.get(k, (0, 0.0))
            out[k] = (n + 1, ms + a.elapsed_time(b))
        return out

    def groups(self):
        """{(kind, masks, table_rows, n_cols, d): [launches, total ms, rows, nnz]}
        over every timed launch (rows / nnz summed over the launches: full-CSR and
        range launches only; masked launches are data-dependent). `masks` names
        the masks a launch was given ("row_list", "row", "src", "src+row"; "" for
        unmasked), so the different frontier products stay apart."""
        torch.cuda.synchronize()
        out = {}
        for rows, nnz, d, m, a, b, tr, nc, sig in self.records:
            g = out.setdefault((m, sig, tr, nc, d), [0, 0.0, 0, 0])
            g[0] += 1
            g[1] += a.elapsed_time(b)
            g[2] += rows
            g[3] += nnz
        return out

    def edge_counts(self):
        """{(kind, masks, table_rows, n_cols, d): [launches, rows, visited, gathered]}
        summed over the counted launches: `visited` = edges of the rows a launch
        computes (index + weight read), `gathered` = those whose source row is
        read and multiply-added (a src_mask skips exact-zero sources)."""
        out = {}
        for kind, sig, tr, nc, d, r, v, g in self.counts:
            e = out.setdefault((kind, sig, tr, nc, d), [0, 0, 0, 0])
            e[0] += 1
            e[1] += int(r)
            e[2] += int(v)
            e[3] += int(g)
        return out

    def sequence(self, kind: str, steps: int):
        """Per-position average ms of one kind of launch within a step (every
        step issues the same launch sequence): [(rows, nnz, avg_ms), ...]."""
        torch.cuda.synchronize()
        recs = [r for r in self.records if r[3] == kind]
        if steps <= 0 or len(recs) % steps:
            return []
        per = len(recs) // steps
        out = []
        for j in range(per):
            ms = sum(recs[s * per + j][4].elapsed_time(recs[s * per + j][5])
                     for s in range(steps)) / steps
            out.append((recs[j][0], recs[j][1], ms))
        return out

    def count_launch(self, prod: "Product", kind: str, d: int, rng, src_mask, row_mask,
                     row_list, src_input: bool = False) -> None:
        """Device-side count of the rows / edges one launch processes (stream-
        ordered torch ops on the launch's own masks, read after the steps)."""
        c = prod.csr
        deg = c.__dict__.get("_deg64")
        if deg is None:
            deg = c.__dict__["_deg64"] = c.degrees().long()
        if row_list is not None:
            sel = torch.zeros(c.n_rows, dtype=torch.bool, device=c.device)
            sel[row_list.long()] = True
        else:
            sel = (torch.ones(c.n_rows, dtype=torch.bool, device=c.device)
                   if row_mask is None else row_mask[:c.n_rows].bool())
            if rng is not None:
                keep = torch.zeros_like(sel)
                keep[rng[0]:rng[1]] = True
                sel = sel & keep
        visited = deg[sel].sum()
        if src_mask is None:
            gathered = visited
        else:
            cols = c.__dict__["_input_indices"] if src_input else c.indices
            live = src_mask[cols[:c.nnz].long()].bool()
            gathered = (live & torch.repeat_interleave(sel, deg)).sum()
        self.counts.append((kind, mask_signature(src_mask, row_mask, row_list), c.n_rows,
                            c.n_cols, d, sel.sum(), visited, gathered))


def mask_signature(src_mask, row_mask, row_list) -> str:
    if row_list is not None:
        return "row_list"
    return "+".join(n for n, m in (("src", src_mask), ("row", row_mask)) if m is not None)


_timer: SpmmTimer | None = None


class ListLength:
    """The length of a row list built on the stream (bbgr_mark_list's device
    count), for spmm(row_count=...). A launch over a device-length list needs
    a grid for the list's capacity (C4: 62.5k short-row workgroups for the
    ~60k-row item frontier; most only read the length and exit, ~60 us of the
    first backward item product). On an eager stream `publish()` copies the
    count to pinned host memory right after the list is built; a launch then
    waits for that copy and passes the exact list, so its grid is the list's.
    The wait comes where the launch is issued — behind the forward's dense
    products, milliseconds of queued GPU work — so the GPU does not idle.
    Inside a graph capture (or before publish / after invalidate) the launch
    keeps the device count. The rows and their arithmetic are the same either
    way (bitwise). BBGR_LIST_HOST=0 keeps the device count always (A/B runs).

    `wait`: whether a consumer may block on the copy. Only where the stream
    holds queued work between the list and its first consumer (the trainer's
    K >= 2 dense forward layers) does the wait cost the GPU nothing; with
    wait=False a consumer takes the published length only if the copy has
    already landed (event query), else the device count."""

    enabled = os.environ.get("BBGR_LIST_HOST", "1") != "0"

    def __init__(self, count: torch.Tensor, wait: bool = True):
        self.count = count
        self.wait = bool(wait)
        self._host = torch.zeros(1, dtype=torch.int64, pin_memory=True)
        self._event = None

    def publish(self) -> None:
        """After the list is built, on the current stream."""
        self._event = None
        if not self.enabled or torch.cuda.is_current_stream_capturing():
            return
        self._host.copy_(self.count, non_blocking=True)
        self._event = torch.cuda.Event()
        self._event.record()

    def invalidate(self) -> None:
        self._event = None

    def length(self) -> int | None:
        """The published length (waiting for its copy when `wait`), or None:
        use the device count."""
        if self._event is None or torch.cuda.is_current_stream_capturing():
            return None
        if not self._event.query():
            if not self.wait:
                return None
            self._event.synchronize()
        return int(self._host[0])


def set_spmm_timer(t: SpmmTimer | None) -> None:
    global _timer
    _timer = t


def spmm(prod: Product, x: torch.Tensor, first: bool, *, y=None, y_scale=None,
         y_scale_s: float = 1.0, add=None, add_scale=None, add_scale_s: float = 1.0,
         acc_in=None, acc_out=None, acc_scale=None, acc_scale_s: float = 1.0,
         gamma: float = 1.0, src_mask=None, row_mask=None, acc_mask=None,
         add_mask=None, row_list=None, rng=None, adam=None, y_map=None, acc_map=None,
         add_map=None, src_input: bool = False, src_bits=None, row_count=None,
         tag_out=None, tag_mask=None, tagged=None, src_mask_bits=None) -> None:
    """One fused SpMM launch (bbgr_spmm) on the current stream. `adam`
    (optim.AdamRows): apply Adam to each row's y value in the epilogue.
    `y_map` / `acc_map` / `add_map`: row maps of those tables (input-order
    tables of a degree-ordered pair); `src_input`: x is gathered through the
    CSR's input-id column indices (Product.input_struct). `src_bits`: the slot
    bitmap of src_mask's live edges in this CSR (bbgr_spmm_args.src_bits).
    `row_count` (device int64): row_list holds that many rows (its numel() is
    the capacity; bbgr_spmm_args.row_count) — a list built on the stream, the
    rows row_mask flags; a ListLength passes the list at its published length
    instead when there is one. `tag_out` / `tag_mask` (a full launch): also
    write the CSR's column indices with bit 31 set where tag_mask is 0;
    `tagged` (with src_mask, the same mask): read liveness from such a copy
    instead of loading src_mask per edge (bbgr_spmm_args.tag_out /
    src_tagged; bitwise the src_mask launch). `src_mask_bits` (with src_mask):
    the same mask packed one bit per row (bbgr_mask_pack), read by the
    per-edge test instead of the bytes (bbgr_spmm_args.src_mask_bits)."""
    listed_on_device = row_count is not None
    if isinstance(row_count, ListLength):
        n = row_count.length()
        if n is None:
            row_count = row_count.count
        else:
            row_list, row_count = row_list[:n], None
    d = x.shape[1]
    a = _lib.SpmmArgs()
    a.d = d
    a.x, a.ldx = ptr(x), ld(x)
    if prod.vals is not None:
        a.weight_mode, a.edge_val = 1, ptr(prod.vals)
    elif first and prod.in_scale is not None:
        a.weight_mode, a.edge_val = 1, ptr(prod.first_layer_values())
    else:
        a.weight_mode = 0
    a.y, a.ldy = ptr(y), ld(y)
    a.y_scale, a.y_scale_s = ptr(y_scale), y_scale_s
    a.add, a.ldadd = ptr(add), ld(add)
    a.add_scale, a.add_scale_s = ptr(add_scale), add_scale_s
    a.acc_in, a.ldacc_in = ptr(acc_in), ld(acc_in)
    a.acc_out, a.ldacc_out = ptr(acc_out), ld(acc_out)
    a.acc_scale, a.acc_scale_s = ptr(acc_scale), acc_scale_s
    a.gamma = gamma
    a.partial = ptr(prod.workspace(d))
    a.src_mask, a.row_mask = ptr(src_mask), ptr(row_mask)
    if tag_out is not None:
        a.tag_out, a.tag_mask = ptr(tag_out), ptr(tag_mask)
    if tagged is not None:
        if src_mask is None:
            raise ValueError("spmm: tagged indices stand for a src_mask; pass it too")
        a.src_tagged, a.src_mask = ptr(tagged), None
    a.acc_mask, a.add_mask = ptr(acc_mask), ptr(add_mask)
    if row_list is not None:
        a.row_list, a.n_row_list = ptr(row_list), row_list.numel()
        if row_count is not None:
            a.row_count = ptr(row_count)
    if rng is not None:   # (row0, row1, chunk0, chunk1, split0, split1): Csr.row_ranges
        a.use_range = 1
        for k in range(6):
            a.range[k] = rng[k]
    if adam is not None:
        adam.fill(a)
    a.y_map, a.acc_map, a.add_map = ptr(y_map), ptr(acc_map), ptr(add_map)
    if src_bits is not None and src_mask is not None:
        a.src_bits = ptr(src_bits)
    if src_mask_bits is not None and a.src_mask:
        a.src_mask_bits = ptr(src_mask_bits)
    # input-order source rows carry no hot prefix; mapped output rows neither
    a.stream_from = 0 if src_input else prod.csr.stream_from(d)
    a.stream_out_from = 0 if y_map is not None else prod.csr.stream_out_from(d)
    cs = prod.input_struct() if src_input else prod.csr._struct
    if _timer is None:
        call("bbgr_spmm", ctypes.byref(cs), ctypes.byref(a), stream_handle())
        return
    masked = src_mask is not None or row_mask is not None or row_list is not None
    kind = "masked" if masked else ("full" if adam is None else
                                    "adam" if adam.grad is None else "adam_side")
    if _timer.select is not None and not _timer.select(kind, prod):
        call("bbgr_spmm", ctypes.byref(cs), ctypes.byref(a), stream_handle())
        return
    if listed_on_device:   # the list is row_mask's rows, built on the stream
        row_list = None
    if _timer.count:
        call("bbgr_spmm", ctypes.byref(cs), ctypes.byref(a), stream_handle())
        _timer.count_launch(prod, kind, d, rng, src_mask, row_mask, row_list, src_input)
        return
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    call("bbgr_spmm", ctypes.byref(cs), ctypes.byref(a), stream_handle())
    ev1.record()
    rows, nnz = prod.csr.n_rows, prod.csr.nnz
    if rng is not None and row_list is None:   # a row range: its own rows and edges
        rows, nnz = rng[1] - rng[0], prod.csr.range_nnz(rng[0], rng[1])
    _timer.records.append((rows, nnz, d, kind, ev0, ev1, prod.csr.n_rows, prod.csr.n_cols,
                           mask_signature(src_mask, row_mask, row_list)))


def epilogue(t: torch.Tensor, *, y=None, y_scale=None, y_scale_s: float = 1.0, add=None,
             add_scale=None, add_scale_s: float = 1.0, acc_in=None, acc_out=None,
             acc_scale=None, acc_scale_s: float = 1.0, gamma: float = 1.0, acc_mask=None,
             add_mask=None, row_mask=None, row_list=None, n_rows: int | None = None) -> None:
    """bbgr_epilogue: the SpMM epilogue applied to a table of row sums: dense
    (row r of t is output row r), or compact with `row_list` (row j of t is
    output row row_list[j]; `n_rows` = the output tables' row count)."""
    a = _lib.SpmmArgs()
    a.d = t.shape[1]
    a.y, a.ldy = ptr(y), ld(y)
    a.y_scale, a.y_scale_s = ptr(y_scale), y_scale_s
    a.add, a.ldadd = ptr(add), ld(add)
    a.add_scale, a.add_scale_s = ptr(add_scale), add_scale_s
    a.acc_in, a.ldacc_in = ptr(acc_in), ld(acc_in)
    a.acc_out, a.ldacc_out = ptr(acc_out), ld(acc_out)
    a.acc_scale, a.acc_scale_s = ptr(acc_scale), acc_scale_s
    a.gamma = gamma
    a.acc_mask, a.add_mask = ptr(acc_mask), ptr(add_mask)
    a.row_mask = ptr(row_mask)
    if row_list is not None:
        if n_rows is None:
            raise ValueError("epilogue: row_list needs n_rows (the output row count)")
        if row_list.numel() > t.shape[0]:
            raise ValueError("epilogue: compact table has fewer rows than row_list")
        a.row_list, a.n_row_list = ptr(row_list), row_list.numel()
    call("bbgr_epilogue", t.shape[0] if n_rows is None else n_rows, ptr(t), ld(t),
         ctypes.byref(a), stream_handle())


def _item_product(prod: Product, x: torch.Tensor, first: bool, reduce, new, **kw) -> None:
    """Item-row product. With a `reduce` hook (user-row sharding), the SpMM writes
    this rank's raw partial row sums, `reduce` sums them over ranks in place
    (RCCL all-reduce), and the epilogue runs on the complete sums."""
    if reduce is None:
        spmm(prod, x, first, **kw)
        return
    for key in ("y_map", "acc_map", "add_map"):   # input-order pairs only
        if kw.pop(key, None) is not None:
            raise ValueError("sharded item products take no input-order maps")
    if kw.pop("src_input", False):
        raise ValueError("sharded item products take no input-order maps")
    if hasattr(reduce, "item_product"):   # chunked / overlapped exchange (takes src_bits)
        reduce.item_product(prod, x, first, new, kw)
        return
    kw.pop("src_bits", None)   # an index-scan shortcut only: the mask alone is exact
    src_mask = kw.pop("src_mask", None)
    row_mask = kw.pop("row_mask", None)
    t = new("partial", prod.csr.n_rows)
    spmm(prod, x, first, y=t, src_mask=src_mask, row_mask=row_mask)
    reduce(t)
    epilogue(t, row_mask=row_mask, **kw)


def _check_table(name, t, rows, d=None):
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    if t.dim() != 2 or t.shape[0] != rows or (d is not None and t.shape[1] != d):
        raise ValueError(f"{name} has shape {tuple(t.shape)}, expected [{rows}, {d}]")
    if t.stride(1) != 1:
        raise ValueError(f"{name} must have unit column stride")


def _buffers(ws: dict | None, device, d: int):
    """Allocator for the chain's intermediate tables; reuses ws[(tag, rows, d)]."""
    def new(tag: str, n: int) -> torch.Tensor:
        if ws is None:
            return torch.empty(n, d, dtype=torch.float32, device=device)
        key = (tag, n, d)
        t = ws.get(key)
        if t is None:
            t = ws[key] = torch.empty(n, d, dtype=torch.float32, device=device)
        return t
    return new


def drain(steps):
    """Run a *_steps generator to its end and return its value."""
    try:
        while True:
            next(steps)
    except StopIteration as stop:
        return stop.value


def forward_steps(pair: OperatorPair, u0: torch.Tensor, i0: torch.Tensor, num_layers: int,
                  order: str = ORDER_GS, out_u: torch.Tensor | None = None,
                  out_i: torch.Tensor | None = None, ws: dict | None = None, reduce=None,
                  final_rows=None, tag=None):
    """Final (layer-mean) user and item tables. u0 [U,d], i0 [I,d] fp32.
    A generator: it yields after issuing each item-row product (with `reduce`,
    each exchange point), so the caller can interleave the issue of several
    chains (ShardedTrainer column chains); `drain()` / `forward()` run it whole.
    `reduce(t)`: in-place sum over ranks of item-row partial sums (sharded mode).
    `final_rows=(user_mask, item_mask[, user_list[, (item_list, item_count)[,
    item_acc_mask]]])`: only the flagged rows of the final
    tables are needed (a training step reads batch rows only). The last layer
    then computes only those rows; the item mask must cover every item the
    flagged users' last-layer rows read (GS: N(batch users) and the batch
    items; Jacobi: the batch items). Flagged rows are bitwise identical to a
    full pass; the others are left stale. The item list (GS, no `reduce`):
    item_mask's rows with their count in device memory (bbgr_mark_list) — the
    last item product visits them instead of testing every row's mask byte.
    `item_acc_mask`: the item rows whose FINAL value is read (the batch items;
    default item_mask): the item layer-mean accumulator is formed on those
    rows only (item_mask must cover them).
    `tag=(tag_out, tag_mask)` (GS, K >= 2): the first user product, a full
    launch, also writes the user CSR's column indices tagged with tag_mask
    (bit 31 = dead item) for backward_steps(tagged=...)."""
    U, I = pair.num_users, pair.num_items
    d = u0.shape[1]
    _check_table("user table", u0, U, d)
    _check_table("item table", i0, I, d)
    acc_u = torch.empty_like(u0, memory_format=torch.contiguous_format) if out_u is None else out_u
    acc_i = torch.empty_like(i0, memory_format=torch.contiguous_format) if out_i is None else out_i
    K = int(num_layers)
    if K == 0:
        acc_u.copy_(u0)
        acc_i.copy_(i0)
        return acc_u, acc_i
    gl = 1.0 / (K + 1)
    FI, FU = pair.fwd_item, pair.fwd_user
    new = _buffers(ws, u0.device, d)
    mu, mi, ulist, ilist, ami = ((tuple(final_rows) + (None, None, None))[:5]
                                 if final_rows is not None else (None,) * 5)
    if ami is None:
        ami = mi
    io = pair.io   # input-order tables over a degree-ordered graph (set_input_order)
    if io is not None and (reduce is not None or final_rows is not None):
        raise ValueError("an input-order pair takes neither a reduce hook nor final_rows")
    # the layer-mean accumulators hold the caller's (input-order) rows: every
    # epilogue places them through the side's map; the first products gather
    # the input-order u0 / i0 through input-id column indices
    am_u, am_i = (io.user_map, io.item_map) if io is not None else (None, None)
    if order == ORDER_GS:
        bufU, bufI = new("u0", U), new("i0", I)
        il = {}
        if ilist is not None and reduce is None and mi is not None:
            il = dict(row_list=ilist[0], row_count=ilist[1])
        for k in range(1, K + 1):
            g = gl if k == K else 1.0
            last = k == K
            _item_product(FI, u0 if k == 1 else bufU, k == 1, reduce, new, y=bufI,
                          y_scale=pair.feed_fwd_iu, acc_in=i0 if k == 1 else acc_i,
                          acc_out=acc_i, acc_scale=FI.out_scale, gamma=g,
                          row_mask=mi if last else None, acc_mask=ami, acc_map=am_i,
                          src_input=io is not None and k == 1, **(il if last else {}))
            yield
            tk = {}
            if tag is not None and k == 1 and not last:
                tk = dict(tag_out=tag[0], tag_mask=tag[1])
            spmm(FU, bufI, False, y=bufU if k < K else None, y_scale=pair.feed_fwd_ui,
                 acc_in=u0 if k == 1 else acc_u, acc_out=acc_u,
                 acc_scale=FU.out_scale, gamma=g, row_mask=mu if last else None,
                 acc_mask=mu, row_list=ulist if last else None, acc_map=am_u, **tk)
    elif order == ORDER_J:
        bufU, bufI = [new("u0", U), new("u1", U)], [new("i0", I), new("i1", I)]
        cur = 0
        for k in range(1, K + 1):
            g = gl if k == K else 1.0
            nxt = 1 - cur
            last = k == K
            _item_product(FI, u0 if k == 1 else bufU[cur], k == 1, reduce, new,
                          y=bufI[nxt] if k < K else None, y_scale=pair.feed_fwd_iu,
                          acc_in=i0 if k == 1 else acc_i, acc_out=acc_i,
                          acc_scale=FI.out_scale, gamma=g, row_mask=mi if last else None,
                          acc_mask=ami, acc_map=am_i, src_input=io is not None and k == 1)
            yield
            spmm(FU, i0 if k == 1 else bufI[cur], k == 1,
                 y=bufU[nxt] if k < K else None, y_scale=pair.feed_fwd_ui,
                 acc_in=u0 if k == 1 else acc_u, acc_out=acc_u,
                 acc_scale=FU.out_scale, gamma=g, row_mask=mu if last else None,
                 acc_mask=mu, row_list=ulist if last else None, acc_map=am_u,
                 src_input=io is not None and k == 1)
            cur = nxt
    else:
        raise ValueError(f"unknown propagation order {order!r}")
    return acc_u, acc_i


def forward(pair: OperatorPair, u0: torch.Tensor, i0: torch.Tensor, num_layers: int,
            order: str = ORDER_GS, out_u: torch.Tensor | None = None,
            out_i: torch.Tensor | None = None, ws: dict | None = None, reduce=None,
            final_rows=None, tag=None):
    """forward_steps run to completion: the final (u, i) tables."""
    return drain(forward_steps(pair, u0, i0, num_layers, order, out_u, out_i, ws, reduce,
                               final_rows, tag))


def backward_steps(pair: OperatorPair, gU: torch.Tensor, gI: torch.Tensor, num_layers: int,
                   order: str = ORDER_GS, out_u: torch.Tensor | None = None,
                   out_i: torch.Tensor | None = None, ws: dict | None = None,
                   grad_i0_dense: bool = True, reduce=None, grad_support=None,
                   adam_u=None, before_last=None, adam_i=None, src_bits=None,
                   frontier_list=None, tagged=None, item_mask_bits=None):
    """Gradients w.r.t. (u0, i0) given dL/d(u_final), dL/d(i_final); a
    generator yielding after each item-row product, like forward_steps.
    `adam_u` (optim.AdamRows) fuses the user-table Adam step into the last
    (user-row) product, which then writes no gradient table (out_u is left
    untouched); `before_last()` runs just before the last products, after
    every other read of gU / gI (the trainer adds the ego-L2 rows there).
    Jacobi order, K >= 2, no `reduce`: `adam_i` fuses the item-table Adam into
    the last item-row product the same way (out_i untouched). Jacobi K == 1
    reads gU / gI as the last products' SOURCE tables: not fusable there.
    GS order, K >= 2, no `reduce`: `adam_i` carrying its own gradient table
    (AdamRows(grad=...): the item weights only feed the layer mean, so their
    gradient is known before the chain) rides on the last item product, a
    dense launch over every item row that still writes its output.
    `grad_support=(user_mask, item_mask)`: gU is zero outside the flagged users
    and, for GS, the first item product's output is zero outside the flagged
    items (GS: batch items and N(batch users); Jacobi: gI's own support). The
    first products of the chain then skip the exact-zero source rows; results
    are bitwise identical to the dense chain (the skipped terms are +0.0).
    `src_bits`: the item-CSR slot bitmap of the flagged users' edges
    (graph.user_item_slots + bbgr_mark_slots): the first item product then
    tests liveness on it instead of scanning every index of its rows.
    `frontier_list=(rows, count)`: GS, no `reduce` — the flagged items as a
    row list of capacity rows.numel() whose length is the device int64 count
    (bbgr_mark_list): the first item product then visits those rows only
    instead of testing every row's mask byte.
    `tagged` (GS): the user CSR's column indices tagged with grad_support's
    item mask (forward_steps(tag=...)): the first user product reads the item
    support from them instead of loading the mask per edge (bitwise).
    `item_mask_bits`: grad_support's item mask packed one bit per item
    (bbgr_mask_pack): the first user product tests its edges on the bits
    instead of the bytes (bitwise; GS and Jacobi, graph-ordered sources)."""
    U, I = pair.num_users, pair.num_items
    d = gU.shape[1]
    _check_table("user grad", gU, U, d)
    _check_table("item grad", gI, I, d)
    K = int(num_layers)
    gu0 = torch.empty_like(gU, memory_format=torch.contiguous_format) if out_u is None else out_u
    gi0 = torch.empty_like(gI, memory_format=torch.contiguous_format) if out_i is None else out_i
    if K == 0:
        gu0.copy_(gU)
        gi0.copy_(gI)
        return gu0, gi0
    gl = 1.0 / (K + 1)
    BI, BU = pair.bwd_item, pair.bwd_user
    new = _buffers(ws, gU.device, d)
    io = pair.io
    if io is not None and reduce is not None:
        raise ValueError("an input-order pair takes no reduce hook")
    # input-order pair: gU / gI / the outputs are in the caller's order (row
    # maps on add / y, input-id gathers in the first products); grad_support
    # is then (su, si, si_internal): su / si index input-order rows (the add
    # tables' and the first products' sources), si_internal the item CSR rows
    if grad_support is None:
        su = si = si_int = None
    elif io is not None:
        su, si, si_int = grad_support
    else:
        su, si = grad_support
        si_int = si
    um, im = (io.user_map, io.item_map) if io is not None else (None, None)
    inp = io is not None
    if order == ORDER_GS:
        bufU, bufI = new("u0", U), new("i0", I)
        fl = {}
        if frontier_list is not None and reduce is None and si_int is not None:
            fl = dict(row_list=frontier_list[0], row_count=frontier_list[1])
        if adam_i is not None and (K < 2 or reduce is not None or adam_i.grad is None):
            raise ValueError("GS backward: a fused item Adam needs K >= 2, no reduce hook "
                             "and its own gradient table (AdamRows(grad=...))")
        for k in range(K, 0, -1):
            first = k == K
            ka = {"adam": adam_i} if (k == 1 and adam_i is not None) else {}
            # first product: Gi_K is zero off the item support (batch items and
            # N(batch users)) and the next product reads only that support, so
            # the other rows are neither computed nor written (row_mask)
            _item_product(BI, gU if first else bufU, first, reduce, new, y=bufI,
                          y_scale=pair.feed_bwd_iu, y_scale_s=gl if first else 1.0,
                          add=gI, add_mask=si, add_scale=BU.in_scale, add_scale_s=gl,
                          src_mask=su if first else None,
                          row_mask=si_int if first else None, add_map=im,
                          src_input=inp and first, src_bits=src_bits if first else None,
                          **(fl if first else {}), **ka)
            yield
            tg = tagged if (first and si_int is not None) else None
            mb = item_mask_bits if (first and si_int is not None and tg is None) else None
            if k > 1:
                spmm(BU, bufI, False, y=bufU, y_scale=pair.feed_bwd_ui,
                     add=gU, add_mask=su, add_scale=BI.in_scale, add_scale_s=gl,
                     src_mask=si_int if first else None, add_map=um, tagged=tg,
                     src_mask_bits=mb)
            else:
                if before_last is not None:
                    before_last()
                src = si_int if first else None
                fused = adam_u is not None and src is None   # fused Adam needs every row
                spmm(BU, bufI, False, y=None if fused else gu0, y_scale=BU.out_scale,
                     add=gU, add_mask=su, add_scale=None, add_scale_s=gl,
                     src_mask=src, adam=adam_u if fused else None, add_map=um, y_map=um,
                     tagged=tg, src_mask_bits=mb)
                if adam_u is not None and not fused:   # K == 1: masked product, Adam apart
                    adam_u.apply(gu0)
        if grad_i0_dense:   # GS: i0 only feeds the layer mean -> grad_i0 = gI/(K+1)
            torch.mul(gI, gl, out=gi0)
    elif order == ORDER_J:
        if (adam_u is not None or adam_i is not None) and (K < 2 or before_last is None):
            raise ValueError("fused Adam in the Jacobi backward needs K >= 2 and before_last")
        if adam_i is not None and reduce is not None:
            raise ValueError("fused item Adam needs the complete item sums (no reduce hook)")
        bufU, bufI = [new("u0", U), new("u1", U)], [new("i0", I), new("i1", I)]
        cur = 0
        for k in range(K, 0, -1):
            first = k == K
            nxt = 1 - cur
            ys = gl if first else 1.0
            xu = gI if first else bufI[cur]   # input of BU (item table)
            xi = gU if first else bufU[cur]   # input of BI (user table)
            mu_ = si if first else None     # BU reads gI (items), BI reads gU (users)
            mi_ = su if first else None
            src_in = inp and first           # gI / gU: input order
            mb = item_mask_bits if (first and mu_ is not None and not src_in) else None
            if k > 1:
                spmm(BU, xu, first, y=bufU[nxt], y_scale=pair.feed_bwd_ui, y_scale_s=ys,
                     add=gU, add_mask=su, add_scale=BI.in_scale, add_scale_s=gl, src_mask=mu_,
                     add_map=um, src_input=src_in, src_mask_bits=mb)
                _item_product(BI, xi, first, reduce, new, y=bufI[nxt],
                              y_scale=pair.feed_bwd_iu, y_scale_s=ys,
                              add=gI, add_mask=si, add_scale=BU.in_scale, add_scale_s=gl,
                              src_mask=mi_, add_map=im, src_input=src_in,
                              src_bits=src_bits if first else None)
                yield
            else:
                if before_last is not None and adam_u is not None:
                    before_last()
                spmm(BU, xu, first, y=None if adam_u is not None else gu0, y_scale=BU.out_scale,
                     y_scale_s=ys, add=gU, add_mask=su, add_scale=None, add_scale_s=gl,
                     src_mask=mu_, adam=adam_u, add_map=um, y_map=um, src_input=src_in,
                     src_mask_bits=mb)
                ik = dict(y=None if adam_i is not None else gi0, y_scale=BI.out_scale,
                          y_scale_s=ys, add=gI, add_mask=si, add_scale=None, add_scale_s=gl,
                          src_mask=mi_, add_map=im, y_map=im, src_input=src_in,
                          src_bits=src_bits if first else None)
                if adam_i is not None:
                    ik["adam"] = adam_i
                _item_product(BI, xi, first, reduce, new, **ik)
                yield
            cur = nxt
    else:
        raise ValueError(f"unknown propagation order {order!r}")
    return gu0, gi0


def backward(pair: OperatorPair, gU: torch.Tensor, gI: torch.Tensor, num_layers: int,
             order: str = ORDER_GS, out_u: torch.Tensor | None = None,
             out_i: torch.Tensor | None = None, ws: dict | None = None,
             grad_i0_dense: bool = True, reduce=None, grad_support=None,
             adam_u=None, before_last=None, adam_i=None, src_bits=None,
             frontier_list=None, tagged=None, item_mask_bits=None):
    """backward_steps run to completion: (grad u0, grad i0)."""
    return drain(backward_steps(pair, gU, gI, num_layers, order, out_u, out_i, ws,
                                grad_i0_dense, reduce, grad_support, adam_u, before_last,
                                adam_i, src_bits, frontier_list, tagged, item_mask_bits))


def propagate(pair: OperatorPair, u0: torch.Tensor, i0: torch.Tensor, num_layers: int,
              order: str = ORDER_GS):
    """Differentiable (u0, i0) -> (u_final, i_final): the registered operator
    bbgr::propagate (ops.py), whose backward is bbgr::propagate_backward;
    replaces the autograd of the reference's K x torch.sparse.mm +
    stack().mean() chain."""
    from . import ops
    return ops.propagate(u0, i0, ops.pair_key(pair), int(num_layers), order)


def propagate_rows(pair: OperatorPair, u0: torch.Tensor, i0: torch.Tensor, num_layers: int,
                   order: str, users: torch.Tensor, items: torch.Tensor):
    """propagate() with the final tables valid at the listed rows only (users,
    items: the caller's row ids; GS order — Jacobi computes every row):
    bbgr::propagate_rows. Its backward is propagate's, so a loss over those
    rows gets the same gradients; the listed rows hold the same bits."""
    from . import ops
    return ops.propagate_rows(u0, i0, users, items, ops.pair_key(pair), int(num_layers), order)


# ---------------------------------------------------------------------------
# Square generic operator (lightgcn.py fed an arbitrary N x N sparse tensor)
# ---------------------------------------------------------------------------
class SquareOperator:
    """x_{k+1} = A x_k with explicit values (A and A^T CSRs)."""

    def __init__(self, A: Csr, At: Csr):
        self.A, self.At = A, At
        self.fwd = Product(A, A.values, None, None, {})
        self.bwd = Product(At, At.values, None, None, {})
        self.n = A.n_rows


def square_forward(op: SquareOperator, x0: torch.Tensor, K: int):
    d = x0.shape[1]
    _check_table("node table", x0, op.n, d)
    out = torch.empty_like(x0, memory_format=torch.contiguous_format)
    if K == 0:
        out.copy_(x0)
        return out
    gl = 1.0 / (K + 1)
    bufs = [torch.empty_like(out), torch.empty_like(out)]
    cur = 0
    for k in range(1, K + 1):
        spmm(op.fwd, x0 if k == 1 else bufs[cur], k == 1, y=bufs[1 - cur] if k < K else None,
             acc_in=x0 if k == 1 else out, acc_out=out, gamma=gl if k == K else 1.0)
        cur = 1 - cur
    return out


def square_backward(op: SquareOperator, g: torch.Tensor, K: int):
    out = torch.empty_like(g, memory_format=torch.contiguous_format)
    if K == 0:
        out.copy_(g)
        return out
    gl = 1.0 / (K + 1)
    # G_k = g' + A^T G_{k+1}, G_K = g'; grad_x0 = G_0
    bufs = [torch.empty_like(out), torch.empty_like(out)]
    cur = 0
    for k in range(K, 0, -1):
        first = k == K
        spmm(op.bwd, g if first else bufs[cur], first,
             y=out if k == 1 else bufs[1 - cur], y_scale_s=gl if first else 1.0,
             add=g, add_scale_s=gl)
        cur = 1 - cur
    return out


class _SquareFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x0, op, K):
        _lib.require_gpu(x0)
        ctx.op, ctx.K = op, K
        return square_forward(op, x0.contiguous(), K)

    @staticmethod
    def backward(ctx, g):
        return square_backward(ctx.op, g.contiguous(), ctx.K), None, None
