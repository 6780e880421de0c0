"""Device CSR structures and the factored bipartite operators.

Every propagation operator of the reference factors over ONE bipartite
adjacency A (user-row CSR ``A_ui`` and its transpose, the item-row CSR
``A_iu``) and four diagonal scale vectors:

    item <- user:  M = diag(p) A_iu diag(q)     user <- item:  M = diag(s) A_ui diag(t)

  * GS  (Version-2/lighgcn_cu_pop.py:429-452):  p = t = b, q = c*a, s = a
  * Method A (version_1/lightgcn_cu_pop_long_tail_exposure.py:362-396):
                                                p = t = b*alpha, q = c*a, s = a
  * J   (lightgcn_cu.py:368-399; same weights, Jacobi layer order)
  * SYM (lightgcn.py:352-372): the N x N symmetric D^-1/2 A D^-1/2 restricted
        to its two off-diagonal blocks: p = t = deg_i^-1/2, q = s = deg_u^-1/2

with a = 1/sqrt(max(deg_u,1)), b = 1/sqrt(max(deg_i,1)), c = credibility.
The backward operators are the transposes, i.e. the same two CSRs with the
roles of the scale vectors swapped — nothing else is stored.

Duplicate (u, i) train pairs stay as repeated CSR entries: the SpMM sums them,
which is what ``sparse_coo_tensor(...).coalesce()`` does with their values
(Version-2/lighgcn_cu_pop.py:443,450; lightgcn_cu.py:393,397; lightgcn.py:363).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_handle

DEFAULT_LONG_THRESHOLD = None   # None: long_threshold_for(nnz)
DEFAULT_CHUNK_EDGES = 2048
# Rows longer than the threshold are cut into chunk workgroups (16 lane groups
# on one row) instead of one lane group walking the row in 16-edge batches.
# On a small graph the longest short row is the launch's critical path: at C2
# (1M edges) the step ran 0.887 ms with 256, 0.710 with 128, 0.579 with 64,
# 0.579 with 32, 0.812 with 16; at C4 (50M) 16.77 / 16.76 / 16.97 ms for
# 256 / 128 / 64 (tools/probes/chunk_probe.py, profiles/round1-2/r15_chunk_probe.jsonl).
SMALL_CSR_EDGES = 8_000_000


def long_threshold_for(nnz: int) -> int:
    return 64 if nnz < SMALL_CSR_EDGES else 256
# Hot-row budget of a gathered table in descending-degree order (per CSR:
# Csr.hot_bytes overrides it; a table within the budget streams nothing): rows past it
# are loaded non-temporal (bbgr_spmm_args.stream_from). Sized to leave room in
# the 256 MB Infinity Cache for the streams of the launch; at most 1/8 of the
# rows (C4: the 625k highest-degree users and 125k items stay cached).
HOT_BYTES = 192 << 20
# Output store policy of degree-ordered tables (A/B runs, BBGR_STREAM_OUT):
# "split" = the hot prefix default-policy, the rest non-temporal (stream_out_from);
# "nt" = every row non-temporal; "none" = every row default-policy.
import os as _os  # noqa: E402
OUT_POLICY = _os.environ.get("BBGR_STREAM_OUT", "split")


def _as_device_i32(x, device) -> torch.Tensor:
    if isinstance(x, np.ndarray) and x.dtype == np.int32 and x.ndim == 1:
        from .ingest import to_device_i32    # chunked, works on memory maps
        return to_device_i32(x, device)
    if isinstance(x, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(x.astype(np.int32, copy=False)))
    else:
        t = torch.as_tensor(x)
    return t.to(device=device, dtype=torch.int32).contiguous()


class Csr:
    """Row-sorted CSR on the device (int32 indptr/indices, columns sorted in
    each row, duplicates kept) plus the SpMM load-balance plan."""

    cols_sorted = True   # columns ascending inside each row (membership searches)

    def __init__(self, rows, cols, n_rows: int, n_cols: int, device,
                 edge_values: torch.Tensor | None = None,
                 long_threshold: int | None = DEFAULT_LONG_THRESHOLD,
                 chunk_edges: int = DEFAULT_CHUNK_EDGES, keep_perm: bool = False):
        _lib.require_gpu()
        device = torch.device(device)
        rows = _as_device_i32(rows, device)
        cols = _as_device_i32(cols, device)
        if rows.numel() != cols.numel():
            raise ValueError("rows and cols must have the same length")
        nnz = rows.numel()
        if nnz >= 2**31 - 1:
            raise ValueError("nnz must be < 2^31 for the int32 CSR")
        if nnz and (int(rows.min()) < 0 or int(rows.max()) >= n_rows
                    or int(cols.min()) < 0 or int(cols.max()) >= n_cols):
            raise ValueError("edge index out of range")
        self.n_rows, self.n_cols, self.nnz = int(n_rows), int(n_cols), int(nnz)
        if long_threshold is None:
            long_threshold = long_threshold_for(self.nnz)
        self.device = device
        self.indptr = torch.empty(self.n_rows + 1, dtype=torch.int32, device=device)
        self.indices = torch.empty(max(nnz, 1), dtype=torch.int32, device=device)
        perm = (torch.empty(max(nnz, 1), dtype=torch.int32, device=device)
                if edge_values is not None or keep_perm else None)
        st = stream_handle()
        ws_bytes = _lib.workspace_query(
            "bbgr_csr_build", nnz, ptr(rows), ptr(cols), self.n_rows, self.n_cols,
            ptr(self.indptr), ptr(self.indices), ptr(perm), args_after=(st,))
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=device)
        n = ctypes.c_size_t(ws_bytes)
        call("bbgr_csr_build", nnz, ptr(rows), ptr(cols), self.n_rows, self.n_cols,
             ptr(self.indptr), ptr(self.indices), ptr(perm), ptr(ws), ctypes.byref(n), st)
        del ws
        self.perm = perm if keep_perm else None   # CSR slot -> input edge id
        self.values = None
        if edge_values is not None:
            ev = torch.as_tensor(edge_values).to(device=device, dtype=torch.float32)
            self.values = ev[perm[:nnz].long()].contiguous() if nnz else ev.new_zeros(1)
        self._plan(long_threshold, chunk_edges)

    def _plan(self, long_threshold: int, chunk_edges: int) -> None:
        s = self.struct(with_plan=False)
        s.long_threshold = long_threshold
        s.chunk_edges = chunk_edges
        st = stream_handle()
        ws_bytes = _lib.workspace_query("bbgr_csr_plan_count", ctypes.byref(s), None,
                                        None, args_after=(st,))
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=self.device)
        nb = ctypes.c_size_t(ws_bytes)
        nc, ns = ctypes.c_int32(0), ctypes.c_int32(0)
        call("bbgr_csr_plan_count", ctypes.byref(s), ctypes.byref(nc), ctypes.byref(ns),
             ptr(ws), ctypes.byref(nb), st)
        self.long_threshold, self.chunk_edges = long_threshold, chunk_edges
        self.n_chunks, self.n_split = nc.value, ns.value
        self.chunks = torch.empty(max(4 * self.n_chunks, 4), dtype=torch.int32,
                                  device=self.device)
        self.split = torch.empty(max(4 * self.n_split, 4), dtype=torch.int32,
                                 device=self.device)
        s.n_chunks, s.n_split = self.n_chunks, self.n_split
        call("bbgr_csr_plan_build", ctypes.byref(s), ptr(self.chunks), ptr(self.split),
             ptr(ws), ctypes.byref(nb), st)
        self._struct = self.struct(with_plan=True)

    def struct(self, with_plan: bool = True) -> _lib.CsrStruct:
        s = _lib.CsrStruct()
        s.n_rows, s.n_cols, s.nnz = self.n_rows, self.n_cols, self.nnz
        s.indptr, s.indices = ptr(self.indptr), ptr(self.indices)
        if with_plan:
            s.long_threshold, s.chunk_edges = self.long_threshold, self.chunk_edges
            s.n_chunks, s.n_split = self.n_chunks, self.n_split
            s.chunks, s.split = ptr(self.chunks), ptr(self.split)
        return s

    def range_nnz(self, r0: int, r1: int) -> int:
        """Edges of rows [r0, r1) (host copy of indptr, made once; timing only)."""
        h = self.__dict__.get("_indptr_host")
        if h is None:
            h = self.__dict__["_indptr_host"] = self.indptr.cpu().numpy().astype(np.int64)
        return int(h[r1] - h[r0])

    def row_ranges(self, parts: int, balance_indptr: torch.Tensor | None = None) -> list:
        """Split rows into `parts` contiguous ranges of ~equal edge counts, each as
        (row0, row1, chunk0, chunk1, split0, split1) for bbgr_spmm's range mode.
        `balance_indptr` (default: this CSR's) sets the row boundaries — sharded
        ranks pass the GLOBAL item indptr so every rank cuts at the same rows.
        One host copy of indptr / plan at first use (setup-time)."""
        key = (int(parts), None if balance_indptr is None else balance_indptr.data_ptr())
        cache = self.__dict__.setdefault("_ranges", {})
        if key in cache:
            return cache[key]
        src = self.indptr if balance_indptr is None else balance_indptr
        indptr = src.cpu().numpy().astype(np.int64)
        total = int(indptr[-1])
        ch_rows = self.chunks[: 4 * self.n_chunks].view(-1, 4)[:, 0].cpu().numpy()
        sp_rows = self.split[: 4 * self.n_split].view(-1, 4)[:, 0].cpu().numpy()
        targets = [total * k // parts for k in range(parts + 1)]
        bounds = np.searchsorted(indptr, targets, side="left")
        bounds[0], bounds[-1] = 0, self.n_rows
        bounds = np.maximum.accumulate(np.minimum(bounds, self.n_rows))
        out = []
        for k in range(parts):
            r0, r1 = int(bounds[k]), int(bounds[k + 1])
            if r1 <= r0:
                continue
            c0, c1 = np.searchsorted(ch_rows, [r0, r1], side="left")
            s0, s1 = np.searchsorted(sp_rows, [r0, r1], side="left")
            out.append((r0, r1, int(c0), int(c1), int(s0), int(s1)))
        cache[key] = out
        return out

    def stream_from(self, d: int) -> int:
        """bbgr_spmm_args.stream_from for a gather of d-wide source rows: 0
        unless the columns are in descending-degree order (BipartiteGraph with
        vertex_order="degree"); then the hot prefix of the source table."""
        if not self.__dict__.get("cols_by_degree", False):
            return 0
        hot = self.__dict__.get("hot_bytes", HOT_BYTES)
        if self.n_cols * 4 * d <= hot:   # the whole table stays cached (C1, C2)
            return 0
        return max(1, min(self.n_cols // 8, hot // (4 * d)))

    def stream_out_from(self, d: int) -> int:
        """bbgr_spmm_args.stream_out_from for d-wide output rows: 0 unless the
        rows are in descending-degree order; then the hot prefix of the output
        table (the next product gathers it)."""
        if not self.__dict__.get("rows_by_degree", False):
            return 0
        hot = self.__dict__.get("hot_bytes", HOT_BYTES)
        if self.n_rows * 4 * d <= hot:
            return 0
        if OUT_POLICY == "nt":      # A/B: every output row streamed
            return 1
        if OUT_POLICY == "none":    # A/B: every output row default policy
            return 0
        return max(1, min(self.n_rows // 8, hot // (4 * d)))

    def partial_workspace(self, d: int) -> torch.Tensor | None:
        """bbgr_spmm_args.partial: n_chunks*d floats of chunk partials, then
        n_chunks int32 arrival counters that must start at zero (every launch
        leaves them zero again)."""
        if self.n_split == 0:
            return None
        return torch.zeros(self.n_chunks * (d + 1), dtype=torch.float32, device=self.device)

    def degrees(self) -> torch.Tensor:
        return (self.indptr[1:] - self.indptr[:-1])

    def nbytes(self) -> int:
        return 4 * (self.indptr.numel() + self.indices.numel())


@dataclass
class Scales:
    """Per-row scale vectors of one operator pair (see module docstring)."""
    kind: int
    p: torch.Tensor   # [I] item rows of item<-user
    q: torch.Tensor   # [U] user cols of item<-user
    s: torch.Tensor   # [U] user rows of user<-item
    t: torch.Tensor   # [I] item cols of user<-item
    pt: torch.Tensor  # [I] p*t
    qs: torch.Tensor  # [U] q*s
    deg_u: torch.Tensor
    deg_i: torch.Tensor


class VertexOrder:
    """A renumbering of one vertex set by descending degree (bbgr_degree_order;
    ties keep ascending id): perm[new] = input id, rank[input id] = new."""

    def __init__(self, degree: torch.Tensor):
        degree = degree.to(torch.int32).contiguous()
        n = degree.numel()
        dev = degree.device
        self.perm = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        self.rank = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        st = stream_handle()
        nb = _lib.workspace_query("bbgr_degree_order", n, ptr(degree), ptr(self.perm),
                                  ptr(self.rank), args_after=(st,))
        ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
        have = ctypes.c_size_t(nb)
        call("bbgr_degree_order", n, ptr(degree), ptr(self.perm), ptr(self.rank), ptr(ws),
             ctypes.byref(have), st)
        self.perm, self.rank = self.perm[:n], self.rank[:n]
        self._perm64 = self.perm.long()
        self._rank64 = self.rank.long()

    def to_internal(self, ids: torch.Tensor) -> torch.Tensor:
        """Input ids -> internal row ids (int64)."""
        return self._rank64[ids.to(self._rank64.device).long()]

    def to_input(self, ids: torch.Tensor) -> torch.Tensor:
        """Internal row ids -> input ids (int64)."""
        return self._perm64[ids.to(self._perm64.device).long()]

    def rows_to_internal(self, table: torch.Tensor) -> torch.Tensor:
        """Rows indexed by input id -> rows in internal order (a copy)."""
        return table.to(self._perm64.device)[self._perm64].contiguous()

    def rows_to_input(self, table: torch.Tensor) -> torch.Tensor:
        """Rows in internal order -> rows indexed by input id (a copy)."""
        return table[self._rank64].contiguous()


def _degree_count(ids: torch.Tensor, n: int) -> torch.Tensor:
    """Exact occurrence counts (bbgr_degree_count_ws: per-XCD counter copies)."""
    deg = torch.empty(max(n, 1), dtype=torch.int32, device=ids.device)
    st = stream_handle()
    nb = _lib.workspace_query("bbgr_degree_count_ws", ids.numel(), ptr(ids), n, ptr(deg),
                              args_after=(st,))
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=ids.device)
    have = ctypes.c_size_t(nb)
    call("bbgr_degree_count_ws", ids.numel(), ptr(ids), n, ptr(deg), ptr(ws),
         ctypes.byref(have), st)
    return deg[:n]


def _non_increasing(deg: torch.Tensor) -> bool:
    """True when a degree vector never increases (one device reduction and a
    host read, at graph build)."""
    if deg.numel() < 2:
        return False
    return bool((deg[1:] <= deg[:-1]).all())


def _relabel(ids: torch.Tensor, order: VertexOrder) -> torch.Tensor:
    out = torch.empty_like(ids)
    call("bbgr_relabel", ids.numel(), ptr(ids), ptr(order.rank), ptr(out), stream_handle())
    return out


class BipartiteGraph:
    """The train edges of one split as two device CSRs (user rows, item rows).

    vertex_order="degree" renumbers users and items by descending degree
    before the build (``user_order`` / ``item_order``: VertexOrder; None in
    input order). Every row-indexed tensor of the graph — scales, CSR rows and
    columns, ids the sampler returns — is then in internal order; the trainers
    map inputs and state_dict() across. `item_degree_hook(deg)` (int32 [I] ->
    int32 [I]) replaces the local item degrees that set the item order — the
    sharded trainer passes an all-reduce so every rank orders items alike."""

    def __init__(self, train_edges_2xE, num_users: int, num_items: int, device,
                 long_threshold: int | None = DEFAULT_LONG_THRESHOLD,
                 chunk_edges: int = DEFAULT_CHUNK_EDGES, vertex_order: str = "input",
                 item_degree_hook=None, input_col_order: bool = False):
        device = torch.device(device)
        if isinstance(train_edges_2xE, tuple):        # graph.py's (u2i_src, u2i_dst)
            src, dst = train_edges_2xE
        else:
            e = train_edges_2xE if isinstance(train_edges_2xE, torch.Tensor) \
                else np.asarray(train_edges_2xE)
            if e.shape[0] != 2:
                raise ValueError("train_edges must have shape [2, E]")
            src, dst = e[0], e[1]
        if len(src) != len(dst):
            raise ValueError("source and destination arrays differ in length")
        u = _as_device_i32(src, device)
        i = _as_device_i32(dst, device)
        self.num_users, self.num_items = int(num_users), int(num_items)
        self.nnz = int(u.numel())
        self.device = device
        if vertex_order not in ("input", "degree"):
            raise ValueError(f"vertex_order must be 'input' or 'degree', not {vertex_order!r}")
        self.vertex_order = vertex_order
        self.user_order = self.item_order = None
        if vertex_order == "degree":
            if self.nnz and (int(u.min()) < 0 or int(u.max()) >= self.num_users
                             or int(i.min()) < 0 or int(i.max()) >= self.num_items):
                raise ValueError("edge index out of range")
            deg_i = _degree_count(i, self.num_items)
            if item_degree_hook is not None:
                deg_i = item_degree_hook(deg_i)
            self.user_order = VertexOrder(_degree_count(u, self.num_users))
            self.item_order = VertexOrder(deg_i)
            u_int, i_int = _relabel(u, self.user_order), _relabel(i, self.item_order)
            if input_col_order:
                # rows renumbered, each row's columns kept in ascending INPUT id
                # (the input-order CSR's slot order, then relabelled): every row
                # sums its edges exactly as the input-order graph does, so the
                # drop-in's results are bitwise those of an input-order build;
                # the input-id copies stay for the products that gather the
                # caller's input-order tables (Product.input_struct)
                self.user_csr = Csr(u_int, i, num_users, num_items, device,
                                    long_threshold=long_threshold, chunk_edges=chunk_edges)
                self.item_csr = Csr(i_int, u, num_items, num_users, device,
                                    long_threshold=long_threshold, chunk_edges=chunk_edges)
                for c, order in ((self.user_csr, self.item_order), (self.item_csr,
                                                                    self.user_order)):
                    c.cols_sorted = False   # (no binary search over these rows)
                    c._input_indices = c.indices.clone()
                    call("bbgr_relabel", c.nnz, ptr(c._input_indices), ptr(order.rank),
                         ptr(c.indices), stream_handle())
            u, i = u_int, i_int
        self._u2i_slots = None
        if not (vertex_order == "degree" and input_col_order):
            self.user_csr = Csr(u, i, num_users, num_items, device,
                                long_threshold=long_threshold, chunk_edges=chunk_edges,
                                keep_perm=True)
            self.item_csr = Csr(i, u, num_items, num_users, device,
                                long_threshold=long_threshold, chunk_edges=chunk_edges,
                                keep_perm=True)
            # the user-CSR slot -> item-CSR slot map from the two builds' sort
            # permutations over the same edge list (user_item_slots); the
            # permutations themselves are dropped
            self._u2i_slots = torch.empty(max(self.nnz, 1), dtype=torch.int32, device=device)
            scratch = torch.empty_like(self._u2i_slots)
            call("bbgr_slots_from_perms", self.nnz, ptr(self.user_csr.perm),
                 ptr(self.item_csr.perm), ptr(self._u2i_slots), ptr(scratch), stream_handle())
            del scratch
            self.user_csr.perm = self.item_csr.perm = None
        if vertex_order == "degree":
            users_ordered = items_ordered = True
        else:
            # ids handed over already in descending-degree order (e.g. by
            # ingest.degree_relabel) get the same hot-prefix / streaming cache
            # policy; it changes no value, only which loads are streamed
            users_ordered = _non_increasing(self.user_csr.degrees())
            items_ordered = _non_increasing(self.item_csr.degrees())
        self.user_csr.rows_by_degree = self.item_csr.cols_by_degree = users_ordered
        self.item_csr.rows_by_degree = self.user_csr.cols_by_degree = items_ordered
        self._scales: dict = {}

    def scales(self, kind: int, cred: torch.Tensor | None = None) -> Scales:
        key = (kind, None if cred is None else cred.data_ptr())
        if key in self._scales:
            return self._scales[key]
        U, I, dev = self.num_users, self.num_items, self.device
        f = lambda n: torch.empty(max(n, 1), dtype=torch.float32, device=dev)  # noqa: E731
        deg_u, deg_i = f(U), f(I)
        p, q, s, t, pt, qs = f(I), f(U), f(U), f(I), f(I), f(U)
        if cred is not None:
            cred = cred.to(device=dev, dtype=torch.float32).contiguous().view(-1)
            if cred.numel() != U:
                raise ValueError(f"credibility vector has {cred.numel()} entries, expected {U}")
        call("bbgr_operator_scales", kind, U, I, ptr(self.user_csr.indptr),
             ptr(self.item_csr.indptr), ptr(cred), ptr(deg_u), ptr(deg_i), ptr(p),
             ptr(q), ptr(s), ptr(t), ptr(pt), ptr(qs), stream_handle())
        sc = Scales(kind, p[:I], q[:U], s[:U], t[:I], pt[:I], qs[:U], deg_u[:U], deg_i[:I])
        sc._cred = cred  # keep alive
        self._scales[key] = sc
        return sc

    def user_item_slots(self) -> torch.Tensor:
        """int32 [nnz]: for every user-CSR slot, the item-CSR slot of the same
        edge (bbgr_slots_from_perms at the CSR build; bbgr_transpose_slots for
        other builds). Feeds the slot bitmap of a batch's user edges
        (bbgr_mark_slots -> bbgr_spmm_args.src_bits)."""
        t = self._u2i_slots   # (built with the CSRs; the input-column-order build
        if t is None:          # falls back to a binary search per edge)
            if not (self.user_csr.cols_sorted and self.item_csr.cols_sorted):
                raise ValueError("user_item_slots needs column-sorted CSR rows")
            t = torch.empty(max(self.nnz, 1), dtype=torch.int32, device=self.device)
            call("bbgr_transpose_slots", ctypes.byref(self.user_csr._struct),
                 ctypes.byref(self.item_csr._struct), ptr(t), stream_handle())
            self._u2i_slots = t
        return t

    def nbytes(self) -> int:
        return self.user_csr.nbytes() + self.item_csr.nbytes()
