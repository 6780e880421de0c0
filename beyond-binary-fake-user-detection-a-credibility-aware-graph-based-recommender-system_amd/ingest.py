"""Edge and credibility ingest for the propagation path.

Formats the reference writes and reads, loaded without copies on the host
(memory maps) and streamed to the device in bounded chunks:

  * train/val/test_edges.npy  int32 [2, E]   Version-2/lighgcn_cu_pop.py:299-301,
                                             read at :761-763
  * u2i_src.mmap / u2i_dst.mmap int32 [E], u2i_attr.mmap float32 [E, 5]
    (verified, rating_align, rating, timestamp_norm, helpful_vote)
                                             graph.py:581-587, keys :430, dtypes :436-437
  * credibility CSV (user_id|user_idx, credibility)   Version-2:166-221 /
    lightgcn_cu.py:305-360: missing users default to 1.0, values clipped to
    [0, 1], any other header raises ValueError
  * credibility .npy (main.py:1006 `credibility_scores_minmax.npy`)

Only numpy / csv loaders that execute nothing from the file are used
(np.load(allow_pickle=False), np.memmap, csv).
"""
from __future__ import annotations

import csv
import os
from pathlib import Path

import numpy as np
import torch

U2I_ATTR_KEYS = ("verified", "rating_align", "rating", "timestamp_norm", "helpful_vote")


def load_edges_npy(path, mmap: bool = True) -> np.ndarray:
    """int32 [2, E] edge array (memory-mapped by default)."""
    e = np.load(path, mmap_mode="r" if mmap else None, allow_pickle=False)
    if e.ndim != 2 or e.shape[0] != 2:
        raise ValueError(f"{path}: expected shape [2, E], got {e.shape}")
    if e.dtype != np.int32:
        raise ValueError(f"{path}: expected int32 edges, got {e.dtype}")
    return e


def load_u2i_memmap(directory, with_attr: bool = False):
    """graph.py's edge memmaps: (src[E], dst[E]) int32 [+ attr[E, 5] float32].
    E is inferred from the file size."""
    d = Path(directory)
    src_p, dst_p = d / "u2i_src.mmap", d / "u2i_dst.mmap"
    nbytes = os.path.getsize(src_p)
    if nbytes % 4 or os.path.getsize(dst_p) != nbytes:
        raise ValueError(f"{d}: u2i_src/u2i_dst sizes do not describe int32 [E] arrays")
    E = nbytes // 4
    src = np.memmap(src_p, dtype=np.int32, mode="r", shape=(E,))
    dst = np.memmap(dst_p, dtype=np.int32, mode="r", shape=(E,))
    if not with_attr:
        return src, dst
    attr_p = d / "u2i_attr.mmap"
    if os.path.getsize(attr_p) != E * len(U2I_ATTR_KEYS) * 4:
        raise ValueError(f"{attr_p}: expected float32 [{E}, {len(U2I_ATTR_KEYS)}]")
    attr = np.memmap(attr_p, dtype=np.float32, mode="r", shape=(E, len(U2I_ATTR_KEYS)))
    return src, dst, attr


def to_device_i32(a: np.ndarray, device, chunk: int = 1 << 26) -> torch.Tensor:
    """Stream a host (possibly memory-mapped) int32 vector to the device in
    chunks of `chunk` elements through one pinned staging buffer."""
    n = int(a.shape[0])
    out = torch.empty(max(n, 1), dtype=torch.int32, device=device)[:n]
    if n == 0:
        return out
    dev = torch.device(device)
    stage = torch.empty(min(chunk, n), dtype=torch.int32,
                        pin_memory=dev.type == "cuda" and torch.cuda.is_available())
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        stage[:m].numpy()[:] = a[s:s + m]
        out[s:s + m].copy_(stage[:m], non_blocking=False)
    return out


def edges_to_device(edges, device):
    """(users, items) int32 device vectors from a [2, E] array or a (src, dst) pair."""
    src, dst = (edges[0], edges[1])
    return to_device_i32(np.asarray(src), device), to_device_i32(np.asarray(dst), device)


def degree_relabel(edges, num_users: int, num_items: int):
    """Renumber users and items by descending degree (ties keep ascending id,
    as BipartiteGraph(vertex_order="degree") orders them) once, at ingest.

    Returns (edges', user_ids, item_ids): int32 [2, E] edges in the new ids,
    and int64 maps new id -> original id (user_ids[new] = old). Per-vertex
    inputs follow as `cred[user_ids]`; tables and id lists of a model trained
    on edges' map back with `table[argsort(user_ids)]` / `user_ids[new]`. The reference's ids are arbitrary index maps built at load
    time, so a caller that can renumber them gets the degree-order gathers
    (hot prefix cached, cold rows streamed: BipartiteGraph detects ordered
    ids) in the drop-in module path too (`dropin_module_step`)."""
    src, dst = np.asarray(edges[0]), np.asarray(edges[1])
    out, maps = [], []
    for ids, n in ((src, num_users), (dst, num_items)):
        if ids.size and (int(ids.min()) < 0 or int(ids.max()) >= n):
            raise ValueError("edge index out of range")
        old = np.argsort(-np.bincount(ids, minlength=n), kind="stable")   # new -> old
        rank = np.empty(n, np.int64)
        rank[old] = np.arange(n)
        out.append(rank[ids].astype(np.int32))
        maps.append(old.astype(np.int64))
    return np.stack(out), maps[0], maps[1]


def load_credibility_csv(path, num_users: int, user2idx: dict | None = None) -> np.ndarray:
    """cred[num_users] float32 in [0, 1]; users absent from the file keep 1.0."""
    cred = np.ones((num_users,), dtype=np.float32)
    p = Path(path)
    if not p.exists():
        return cred
    with open(p, "r", encoding="utf-8") as f:
        reader = csv.DictReader(f)
        cols = set(reader.fieldnames or [])
        if "user_id" in cols and "credibility" in cols and user2idx is not None:
            for row in reader:
                uidx = user2idx.get(row.get("user_id") or "")
                if uidx is None:
                    continue
                try:
                    cred[uidx] = float(row["credibility"])
                except (TypeError, ValueError):
                    continue
        elif "user_idx" in cols and "credibility" in cols:
            for row in reader:
                try:
                    u = int(row["user_idx"])
                    if 0 <= u < num_users:
                        cred[u] = float(row["credibility"])
                except (TypeError, ValueError):
                    continue
        else:
            raise ValueError(
                f"[CRED] Unsupported cred CSV header: {reader.fieldnames}. "
                f"Expected (user_id,credibility) OR (user_idx,credibility).")
    return np.clip(cred, 0.0, 1.0).astype(np.float32)


def load_credibility_npy(path, num_users: int | None = None) -> np.ndarray:
    c = np.load(path, allow_pickle=False).astype(np.float32).reshape(-1)
    if num_users is not None and c.size != num_users:
        raise ValueError(f"{path}: {c.size} scores for {num_users} users")
    return np.clip(c, 0.0, 1.0)
