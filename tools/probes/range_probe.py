"""Probe: what a range-pipelined item product costs on one GPU (C4, d=64).

The sharded step cuts each dense item-row product into `parts` row ranges so
range c's all-reduce overlaps range c+1's SpMM. This times one item product:
  one      a single full-CSR launch
  ranges   `parts` range launches back to back (kernel ramp / tail cost)
  events   + an event record after every range (the ordering packet torch's
           async collective puts on the compute stream)
  rccl     + an async all-reduce of the range (world size 1 over RCCL)

    python tools/probes/range_probe.py [--parts 8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import bbgr  # noqa: E402,F401
from bbgr.graph import BipartiteGraph  # noqa: E402
from bbgr.propagate import Product, spmm  # noqa: E402
from bbgr.synthetic import CONFIGS, config_edges  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--hp", action="store_true", help="high-priority RCCL stream")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29583")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    torch.cuda.set_device(0)
    opts = None
    if a.hp:
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0), pg_options=opts)
    c = CONFIGS["C4"]
    g = BipartiteGraph(config_edges("C4"), c["num_users"], c["num_items"], "cuda",
                       vertex_order="degree")
    csr = g.item_csr
    prod = Product(csr, None, None, None, {})
    x = torch.randn(c["num_users"], 64, device="cuda")
    y = torch.empty(c["num_items"], 64, device="cuda")
    rgs = csr.row_ranges(a.parts)

    def one():
        spmm(prod, x, False, y=y)

    side = torch.cuda.Stream()

    def ranges(mode):
        works = []
        for rg in rgs:
            spmm(prod, x, False, y=y, rng=rg)
            if mode == "events":
                torch.cuda.Event().record()
            elif mode == "rccl":
                works.append(dist.all_reduce(y[rg[0]:rg[1]], async_op=True))
            elif mode == "rccl_side":    # collective issued from a side stream
                ev = torch.cuda.Event()
                ev.record()
                with torch.cuda.stream(side):
                    side.wait_event(ev)
                    works.append(dist.all_reduce(y[rg[0]:rg[1]], async_op=True))
        if mode == "rccl_end":
            works.append(dist.all_reduce(y, async_op=True))
        for w in works:
            w.wait()
        if mode == "rccl_side":
            torch.cuda.current_stream().wait_stream(side)

    cases = {"one": one, "ranges": lambda: ranges("plain"), "events": lambda: ranges("events"),
             "rccl": lambda: ranges("rccl"), "rccl_side": lambda: ranges("rccl_side"),
             "rccl_end": lambda: ranges("rccl_end")}
    out = {"parts": len(rgs), "hp": a.hp, "hwq": os.environ.get("GPU_MAX_HW_QUEUES")}
    for name, fn in cases.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            fn()
        torch.cuda.synchronize()
        out[name + "_ms"] = round(1000 * (time.perf_counter() - t0) / a.reps, 4)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()                               # host issue time of one rep, GPU idle
        out[name + "_issue_ms"] = round(1000 * (time.perf_counter() - t0), 4)
        torch.cuda.synchronize()
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
