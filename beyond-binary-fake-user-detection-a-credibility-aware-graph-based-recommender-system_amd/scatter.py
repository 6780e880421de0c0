"""Deterministic row scatter-add (bbgr_scatter_add_rows).

The device form of ``dst.index_add_(0, index, src)`` — the scatter the
reference gets from autograd for the BPR gather (Version-2/lighgcn_cu_pop.py:
495-508 backward) and calls explicitly in the credibility GNN
(main.py:645-650, ``scatter_add``). Unlike an atomic scatter, the addends of
each destination row are summed in ascending source order and added once, so
results are bitwise reproducible.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import call, ld, ptr, stream_handle


class RowScatter:
    """Reusable workspace for bbgr_scatter_add_rows (grown on demand)."""

    def __init__(self):
        self._ws = None

    def __call__(self, dst: torch.Tensor, index: torch.Tensor, src: torch.Tensor,
                 unique: bool = False) -> torch.Tensor:
        """unique=True: the caller guarantees distinct indices (a batch of
        distinct users): one launch, bitwise the sorted path
        (bbgr_rows_add_unique)."""
        _lib.require_gpu(dst)
        n = index.numel()
        if src.shape[0] < n or src.shape[1] != dst.shape[1]:
            raise ValueError("index_add_rows: src must have >= len(index) rows of dst's width")
        for t in (dst, src):
            if not (t.dtype == torch.float32 and t.stride(1) == 1):
                raise ValueError("index_add_rows: fp32 row-major tables")
        index = index.to(torch.int64).contiguous()
        if unique:
            call("bbgr_rows_add_unique", n, ptr(index), ptr(src), ld(src), ptr(dst), ld(dst),
                 dst.shape[1], dst.shape[0], stream_handle())
            return dst
        need = ctypes.c_size_t(0)
        args = (n, ptr(index), ptr(src), ld(src), ptr(dst), ld(dst), dst.shape[1], dst.shape[0])
        call("bbgr_scatter_add_rows", *args, None, ctypes.byref(need), stream_handle())
        if self._ws is None or self._ws.numel() < need.value:
            self._ws = torch.empty(max(need.value, 1), dtype=torch.uint8, device=dst.device)
        have = ctypes.c_size_t(self._ws.numel())
        call("bbgr_scatter_add_rows", *args, ptr(self._ws), ctypes.byref(have), stream_handle())
        return dst


_default = None


def index_add_rows(dst: torch.Tensor, index: torch.Tensor, src: torch.Tensor) -> torch.Tensor:
    """dst.index_add_(0, index, src), deterministic; returns dst."""
    global _default
    if _default is None:
        _default = RowScatter()
    return _default(dst, index, src)
