"""Probe: one middle-layer forward user product of the C4 graph (5M user rows,
user <- item, layer-mean accumulator in place), degree-ordered rows, with each
row's columns (a) in ascending internal (degree-rank) id — the trainer's CSR
— and (b) in ascending INPUT id — the drop-in's CSR, kept so its sums run in
the input-order graph's edge order. Also the middle item product. HIP events
over repeated launches.

    python tools/probes/colorder_probe.py [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bbgr  # noqa: E402,F401
from bbgr._lib import OP_GS  # noqa: E402
from bbgr.graph import BipartiteGraph  # noqa: E402
from bbgr.propagate import OperatorPair, spmm  # noqa: E402
from bbgr.synthetic import CONFIGS, CONFIG_SEED, config_edges, synthetic_credibility  # noqa: E402


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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--warm", type=int, default=1, help="untimed forwards before the timed ones")
    ap.add_argument("--only", default="", choices=["", "trainer", "dropin_py", "env8"],
                    help="just this whole-forward leg, first thing in the process")
    a = ap.parse_args()
    c = CONFIGS["C4"]
    U, I, d = c["num_users"], c["num_items"], c["emb_dim"]
    e = config_edges("C4")
    cred = torch.as_tensor(synthetic_credibility(U, CONFIG_SEED["C4"])).cuda()
    out = {}
    g = torch.Generator(device="cuda").manual_seed(0)
    if not a.only:
        bufI = torch.randn(I, d, device="cuda", generator=g)
        bufU = torch.randn(U, d, device="cuda", generator=g)
        yU, accU = torch.empty(U, d, device="cuda"), torch.randn(U, d, device="cuda", generator=g)
        yI, accI = torch.empty(I, d, device="cuda"), torch.randn(I, d, device="cuda", generator=g)
    for name, inp in (() if a.only else (("sorted", False), ("input_cols", True))):
        gr = BipartiteGraph(e, U, I, "cuda", vertex_order="degree", input_col_order=inp)
        cr = cred[gr.user_order._perm64].contiguous()
        pair = OperatorPair.factored(gr, gr.scales(OP_GS, cr))
        FU, FI = pair.fwd_user, pair.fwd_item
        out[name + "_user_ms"] = timed(lambda: spmm(
            FU, bufI, False, y=yU, y_scale=pair.feed_fwd_ui, acc_in=accU, acc_out=accU,
            acc_scale=FU.out_scale), a.reps)
        out[name + "_item_ms"] = timed(lambda: spmm(
            FI, bufU, False, y=yI, y_scale=pair.feed_fwd_iu, acc_in=accI, acc_out=accI,
            acc_scale=FI.out_scale), a.reps)
        del gr, pair, FU, FI
        torch.cuda.empty_cache()
    # whole forwards, each launch timed: the trainer's pair (sorted columns,
    # internal-order tables) and the drop-in's (input-id columns, input-order
    # tables and maps), in one process
    from bbgr.operators import build_pair
    from bbgr.propagate import SpmmTimer, forward, set_spmm_timer
    from bbgr.trainer import FusedTrainer
    u0 = torch.randn(U, d, device="cuda", generator=g) * 0.01
    i0 = torch.randn(I, d, device="cuda", generator=g) * 0.01
    if not a.only:
        del bufI, bufU, yU, accU, yI, accI
    legs = []
    if a.only in ("", "trainer"):
        tr = FusedTrainer(BipartiteGraph(e, U, I, "cuda", vertex_order="degree"), "v2_pop",
                          cred=cred.cpu().numpy(), emb_dim=d, num_layers=3, batch_size=8192)
        legs.append(("trainer", lambda: forward(tr.pair, tr.user_w, tr.item_w, 3, "gs",
                                                out_u=tr.uf, out_i=tr.itf, ws=tr.ws)))
        legs.append(("trainer_step", tr.step))
    if a.only in ("", "dropin_py"):
        _, _, dpair = build_pair(e, U, I, OP_GS, cred, "cuda")
        legs.append(("dropin_py", lambda: forward(dpair, u0, i0, 3, "gs")))
    for name, run in legs:
        for _ in range(a.warm):   # clocks / power state: a long warm-up first
            run()
        t = SpmmTimer()
        set_spmm_timer(t)
        for _ in range(5):
            run()
        set_spmm_timer(None)
        torch.cuda.synchronize()
        per = len(t.records) // 5
        out[name + "_launch_ms"] = [round(sum(t.records[s * per + j][4].elapsed_time(
            t.records[s * per + j][5]) for s in range(5)) / 5, 3) for j in range(per)]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
