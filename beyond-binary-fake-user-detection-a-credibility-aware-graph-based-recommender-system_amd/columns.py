"""Column-sharded (embedding-dimension) multi-GPU training step.

LightGCN's propagation is linear and acts on every embedding column alike:
column c of each layer depends only on column c of the previous layer
(Version-2/lighgcn_cu_pop.py:482-484 — `torch.sparse.mm(M, E)` is column by
column). So N ranks can each hold ALL users and items, the whole graph, and
d/N of the columns, and run the full K-layer forward, backward and Adam on
their slice with no exchange at all. The only coupling across columns is the
BPR dot products and the ego-L2 norms (:496-507): per triple every rank
computes its share of (s+, s-, |e|^2) — 12 bytes — one all-reduce sums them,
and the loss and every gradient coefficient follow from the complete sums on
every rank (bbgr_bpr's scores_out / scores phases). Batches, negatives and
frontier masks are drawn identically on every rank (same seeds, same graph).

Against the user-row partition (`distributed.ShardedTrainer`) this trades
communication for replicated index traffic: per step each rank reads every
CSR index (12 x 200 MB at C4) but gathers only d/N columns of each source
row, and exchanges 12 B per triple instead of 2(K-1) x I x d x 4 bytes of item
sums (4 x 256 MB at C4). DESIGN §6 has the measured per-rank step for
N = 2, 4, 8 and the comparison.

Column slices must be 8, 16, 32, 64, 128 or 256 wide (narrow rows run the
d/4-lanes-per-row SpMM form, include/bbgr.h).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.distributed as dist

from ._lib import call, stream_handle
from .bpr import bpr_args
from .graph import BipartiteGraph
from .trainer import FusedTrainer

WIDTHS = (8, 16, 32, 64, 128, 256)


def column_range(emb_dim: int, parts: int, index: int) -> tuple[int, int]:
    """Columns [c0, c1) of shard `index` of `parts` (equal widths)."""
    if parts < 1 or emb_dim % parts or not 0 <= index < parts:
        raise ValueError(f"cannot cut {emb_dim} columns into {parts} equal shards")
    w = emb_dim // parts
    if w not in WIDTHS:
        raise ValueError(f"column shard width {w} not in {WIDTHS}")
    return index * w, (index + 1) * w


# Narrowest column shard the bench's auto partition picks: random gathers of
# rows under 64 B (16 fp32 columns) fetch whole cache lines for a fraction of
# them. Measured per-rank C4 steps (one shard alone, tools/probes/column_probe.py,
# profiles/round1-2/r23_*, r32_*): 32 columns 9.05 ms, 16 columns 7.85 ms, 8 columns 7.76 ms
# (the 8-column item product fetches ~3.7x its bytes); single GPU 16.7 ms.
MIN_AUTO_WIDTH = 16


def can_shard_columns(emb_dim: int, parts: int, min_width: int = 8) -> bool:
    return (parts >= 1 and emb_dim % parts == 0 and emb_dim // parts in WIDTHS
            and emb_dim // parts >= min_width)


class ColumnShardedTrainer(FusedTrainer):
    """FusedTrainer on columns [c0, c1) of the embedding tables (see module
    docstring). Every rank passes the same arguments (the whole graph, the
    full-width u0 / i0 or none, the GLOBAL batch size); `group` is the column
    group. Without a process group, `column_parts` / `column_index` build one
    shard alone (a single-GPU stand-in for one rank: its step is the rank's
    work minus the 12-byte score all-reduce, and its loss is that shard's
    partial, not the model's)."""

    def __init__(self, train_edges, num_users: int, num_items: int, variant: str = "v2_pop",
                 cred=None, emb_dim: int = 64, num_layers: int = 3, batch_size: int = 8192,
                 device=None, group=None, u0=None, i0=None, seed: int = 42,
                 vertex_order: str = "degree", column_parts: int | None = None,
                 column_index: int | None = None, **kw):
        self.group = group
        self.distributed = dist.is_available() and dist.is_initialized() and column_parts is None
        if self.distributed:
            self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        else:
            self.world = int(column_parts or 1)
            self.rank = int(column_index or 0)
        self.full_dim = int(emb_dim)
        self.c0, self.c1 = column_range(self.full_dim, self.world, self.rank)
        dev = torch.device(device) if device is not None else torch.device("cuda")
        graph = train_edges if isinstance(train_edges, BipartiteGraph) else \
            BipartiteGraph(train_edges, num_users, num_items, dev, vertex_order=vertex_order)
        if u0 is None:   # FusedTrainer's full-width init (same stream on every rank)
            g = torch.Generator(device="cpu").manual_seed(seed)
            au = (6.0 / (num_users + emb_dim)) ** 0.5
            ai = (6.0 / (num_items + emb_dim)) ** 0.5
            u0 = (torch.rand(num_users, emb_dim, generator=g) * 2 - 1) * au
            i0 = (torch.rand(num_items, emb_dim, generator=g) * 2 - 1) * ai
        u0 = torch.as_tensor(np.asarray(u0) if not isinstance(u0, torch.Tensor) else u0)
        i0 = torch.as_tensor(np.asarray(i0) if not isinstance(i0, torch.Tensor) else i0)
        super().__init__(graph, variant, cred=cred, emb_dim=self.c1 - self.c0,
                         num_layers=num_layers, batch_size=batch_size, seed=seed,
                         u0=u0[:, self.c0:self.c1].contiguous(),
                         i0=i0[:, self.c0:self.c1].contiguous(), **kw)
        self.scores = torch.empty(3 * batch_size, dtype=torch.float32, device=dev)

    def _bpr(self, users, pos, neg, B: int) -> None:
        """Two-phase BPR: this shard's (s+, s-, |e|^2) per triple, summed over
        the column group (12 B per triple), then the loss parts and this
        shard's gradient rows from the complete sums."""
        st = stream_handle()
        sc = self.scores[: 3 * B]
        a = bpr_args(users, pos, neg, self.uf, self.itf, self.user_w, self.item_w, self.reg,
                     self.pop, self.lambda_fair, scores_out=sc)
        call("bbgr_bpr", ctypes.byref(a), st)
        if self.distributed and self.world > 1:
            dist.all_reduce(sc, op=dist.ReduceOp.SUM, group=self.group)
        a = bpr_args(users, pos, neg, self.uf, self.itf, self.user_w, self.item_w, self.reg,
                     self.pop, self.lambda_fair, parts=self.parts[: 3 * B],
                     contrib=self.contrib, scores=sc)
        call("bbgr_bpr", ctypes.byref(a), st)

    def close(self) -> None:
        """Nothing to release (the sharded trainers' close() interface)."""

    def gather_columns(self, t: torch.Tensor) -> torch.Tensor:
        """The full-width table from every rank's column slice (collective)."""
        if not (self.distributed and self.world > 1):
            return t
        parts = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t.contiguous(), group=self.group)
        return torch.cat(parts, dim=1)

    def full_state_dict(self) -> dict:
        """state_dict() at full width (reference keys; collective)."""
        sd = self.state_dict()
        return {k: self.gather_columns(v) for k, v in sd.items()}
