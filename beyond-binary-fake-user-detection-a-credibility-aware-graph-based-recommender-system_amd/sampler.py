"""Batched GPU positive / negative samplers.

Device form of the reference's per-user host loop
(Version-2/lighgcn_cu_pop.py:835-849):
  * sample_pos_item           :339-343  (uniform pick inside the user's row)
  * sample_neg_item_popmix    :349-376  (<= max_tries draws, each from
                              pop_prob with probability mix_pop else uniform,
                              rejected if user_has_item (:330-336); then
                              uniform draws until a non-positive is found)
  * sample_neg_item (uniform) lightgcn.py:296-300 / lightgcn_cu.py:295-299
  * pop_prob = (deg_i+1)^gamma / (sum + 1e-12)  Version-2:805-810, searched
    like numpy's Generator.choice(p=...) (normalised CDF, side='right').

Streams are Philox4x32-10 (key = seed, counter = (draw, slot, step)), so a
(seed, step) pair reproduces a batch exactly; numpy's PCG64 stream is NOT
reproduced ("Sampler parity").
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import call, ptr, stream_handle
from .graph import Csr


class PopMixSampler:
    """Positive + pop-mix negative sampler over a user-row CSR.

    mix_pop = 0 (or gamma=None) gives the uniform sampler of lightgcn.py.
    """

    def __init__(self, user_csr: Csr, item_csr: Csr | None, num_items: int,
                 mix_pop: float = 0.7, gamma: float | None = 0.75, max_tries: int = 50,
                 seed: int = 42):
        _lib.require_gpu()
        if not user_csr.cols_sorted:
            raise ValueError("the sampler's membership search needs column-sorted CSR rows")
        self.csr = user_csr
        self.num_items = int(num_items)
        self.mix_pop = float(mix_pop)
        self.max_tries = int(max_tries)
        self.seed = int(seed)
        self.counter = 0
        self.fail_count = torch.zeros(1, dtype=torch.int32, device=user_csr.device)
        self.cdf = None
        if gamma is not None and mix_pop > 0.0:
            if item_csr is None:
                raise ValueError("pop-mix sampling needs the item-row CSR (item degrees)")
            self.cdf = torch.empty(self.num_items, dtype=torch.float64, device=user_csr.device)
            st = stream_handle()
            nb = _lib.workspace_query("bbgr_pop_cdf", self.num_items, ptr(item_csr.indptr),
                                      float(gamma), ptr(self.cdf), args_after=(st,))
            ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=user_csr.device)
            n = ctypes.c_size_t(nb)
            call("bbgr_pop_cdf", self.num_items, ptr(item_csr.indptr), float(gamma),
                 ptr(self.cdf), ptr(ws), ctypes.byref(n), st)

    def sample(self, users: torch.Tensor, pos: torch.Tensor | None = None,
               neg: torch.Tensor | None = None, counter: int | None = None,
               state: torch.Tensor | None = None):
        """(pos[B], neg[B]) int64 for int64 users[B] (device). `state`: the
        device step state (optim.DeviceStepState.state) whose [1] is this
        step's counter (graph-captured steps); the host counter still advances."""
        users = users.to(dtype=torch.int64).contiguous()
        B = users.numel()
        pos = torch.empty(B, dtype=torch.int64, device=users.device) if pos is None else pos
        neg = torch.empty(B, dtype=torch.int64, device=users.device) if neg is None else neg
        if state is not None:
            self.counter += 1
            call("bbgr_sample_dev", B, ptr(users), ptr(self.csr.indptr), ptr(self.csr.indices),
                 self.num_items, ptr(self.cdf), self.mix_pop, self.max_tries, self.seed,
                 ptr(state), ptr(pos), ptr(neg), ptr(self.fail_count), stream_handle())
            return pos, neg
        c = self.counter if counter is None else int(counter)
        if counter is None:
            self.counter += 1
        call("bbgr_sample", B, ptr(users), ptr(self.csr.indptr), ptr(self.csr.indices),
             self.num_items, ptr(self.cdf), self.mix_pop, self.max_tries, self.seed, c,
             ptr(pos), ptr(neg), ptr(self.fail_count), stream_handle())
        return pos, neg


def shuffle(values: torch.Tensor, seed: int, counter: int, out: torch.Tensor | None = None):
    """Random permutation of an int64 device vector (rng.shuffle, Version-2:821)."""
    values = values.to(dtype=torch.int64).contiguous()
    n = values.numel()
    out = torch.empty_like(values) if out is None else out
    st = stream_handle()
    nb = _lib.workspace_query("bbgr_shuffle", n, ptr(values), ptr(out), seed, counter,
                              args_after=(st,))
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=values.device)
    b = ctypes.c_size_t(nb)
    call("bbgr_shuffle", n, ptr(values), ptr(out), seed, counter, ptr(ws), ctypes.byref(b), st)
    return out


def nonempty_rows(csr: Csr) -> torch.Tensor:
    """Rows with >= 1 edge, ascending (train_users, Version-2:797-798)."""
    st = stream_handle()
    out = torch.empty(max(csr.n_rows, 1), dtype=torch.int64, device=csr.device)
    count = torch.zeros(1, dtype=torch.int64, device=csr.device)
    nb = _lib.workspace_query("bbgr_nonempty_rows", csr.n_rows, ptr(csr.indptr), ptr(out),
                              ptr(count), args_after=(st,))
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=csr.device)
    b = ctypes.c_size_t(nb)
    call("bbgr_nonempty_rows", csr.n_rows, ptr(csr.indptr), ptr(out), ptr(count), ptr(ws),
         ctypes.byref(b), st)
    return out[: int(count.item())]
