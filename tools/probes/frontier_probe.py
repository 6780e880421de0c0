"""Probe: the first backward item product of the C4 step (item <- user, src
mask = the batch users, row mask = the item frontier) in isolation, timed with
HIP events over repeated launches, in forms that give the same rows:

  mask_*      every item row's group tests row_mask
  list_bits   the frontier from a row list of host-known length
  devlist_*   the frontier list with its length in device memory (row_count,
              capacity I: the trainer's form, capturable)
  *_bits      liveness from the slot bitmap (spmm_bits_kernel); *_nobits the mask

Each form's frontier rows are checked bitwise against mask_nobits.

    python tools/probes/frontier_probe.py [--reps 50]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bbgr  # noqa: E402,F401
from bbgr._lib import call, ptr, stream_handle  # noqa: E402
from bbgr.graph import BipartiteGraph  # noqa: E402
from bbgr.propagate import spmm  # noqa: E402
from bbgr.synthetic import CONFIGS, CONFIG_SEED, config_edges, synthetic_credibility  # noqa: E402
from bbgr.trainer import FusedTrainer  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    c = CONFIGS["C4"]
    U, I, d, K, B = (c[k] for k in ("num_users", "num_items", "emb_dim", "num_layers", "batch"))
    e = config_edges("C4")
    tr = FusedTrainer(BipartiteGraph(e, U, I, "cuda", vertex_order="degree"), "v2_pop",
                      cred=synthetic_credibility(U, CONFIG_SEED["C4"]), emb_dim=d,
                      num_layers=K, batch_size=B)
    del e
    tr.step()
    users = tr.next_users()
    pos, neg = tr.sampler.sample(users, tr.posneg[:B], tr.posneg[B:2 * B])
    su, si = tr._set_masks(users, pos, neg, 1)
    g = torch.Generator(device="cuda").manual_seed(1)
    gU = torch.zeros(U, d, device="cuda")
    gI = torch.zeros(I, d, device="cuda")
    gU[users] = torch.randn(B, d, device="cuda", generator=g)
    gI[tr.posneg[:2 * B]] = torch.randn(2 * B, d, device="cuda", generator=g)
    pair = tr.pair
    BI, BU = pair.bwd_item, pair.bwd_user
    gl = 1.0 / (K + 1)
    kw = dict(y_scale=pair.feed_bwd_iu, y_scale_s=gl, add=gI, add_mask=si,
              add_scale=BU.in_scale, add_scale_s=gl, src_mask=su, row_mask=si,
              src_bits=tr.slot_bits)
    lst = torch.empty(I, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    need = ctypes.c_size_t(0)
    call("bbgr_mask_to_list", I, ptr(si), ptr(lst), ptr(cnt), None, ctypes.byref(need),
         stream_handle())
    ws = torch.empty(max(need.value, 1), dtype=torch.uint8, device="cuda")
    call("bbgr_mask_to_list", I, ptr(si), ptr(lst), ptr(cnt), ptr(ws), ctypes.byref(need),
         stream_handle())
    n = int(cnt.item())
    rows = lst[:n]
    csr = BI.csr
    deg = (csr.indptr[1:] - csr.indptr[:-1]).long()
    y_ref = torch.zeros(I, d, device="cuda")
    y = torch.zeros(I, d, device="cuda")
    out = {"frontier_rows": n, "long_rows": int((deg[rows] > csr.long_threshold).sum()),
           "n_chunks": csr.n_chunks,
           "live_edges": int(tr.graph.user_csr.degrees()[users].sum())}
    nobits = dict(kw, src_bits=None)
    forms = {
        "mask_nobits": lambda: spmm(BI, gU, True, y=y, **nobits),
        "mask_bits": lambda: spmm(BI, gU, True, y=y, **kw),
        "list_bits": lambda: spmm(BI, gU, True, y=y, row_list=rows, **kw),
        "devlist_bits": lambda: spmm(BI, gU, True, y=y, row_list=lst, row_count=cnt, **kw),
        "devlist_nobits": lambda: spmm(BI, gU, True, y=y, row_list=lst, row_count=cnt,
                                       **nobits),
    }
    # components (not full results): the multi-chunk rows' workgroups alone
    # (empty list), and the list without its long rows
    zero = torch.zeros(1, dtype=torch.int64, device="cuda")
    short = rows[deg[rows] <= csr.long_threshold]
    out["chunks_only_ms"] = timed(lambda: spmm(BI, gU, True, y=y, row_list=lst, row_count=zero,
                                               **kw), a.reps)
    # the multi-chunk rows' workgroups alone, launched as a range (degree
    # order: those rows come first, their chunks [0, n_multi))
    nch = ((deg + csr.chunk_edges - 1) // csr.chunk_edges) * (deg > csr.long_threshold)
    r1 = int((nch > 1).sum())
    c1 = int(nch[:r1].sum())
    out["multi_rows"], out["multi_chunks"] = r1, c1
    out["multi_range_ms"] = timed(lambda: spmm(BI, gU, True, y=y, row_list=lst, row_count=zero,
                                               rng=(0, r1, 0, c1, 0, csr.n_split), **kw),
                                  a.reps)
    out["short_list_ms"] = timed(lambda: spmm(BI, gU, True, y=y, row_list=short, **kw), a.reps)
    spmm(BI, gU, True, y=y_ref, **nobits)
    for name, fn in forms.items():
        out[name + "_ms"] = timed(fn, a.reps)
        y.zero_()
        fn()
        torch.cuda.synchronize()
        out[name + "_bitwise"] = bool(torch.equal(y[rows], y_ref[rows]))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
