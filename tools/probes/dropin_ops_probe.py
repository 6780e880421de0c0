"""Probe: which torch ops of an eager drop-in step (propagate, bpr_loss,
zero_grad, backward, FusedAdam.step; Version-2/lighgcn_cu_pop.py:858-863)
launch copies or elementwise kernels besides the bbgr operators. One step on
a mid-size Zipf graph under torch.profiler; prints the aten ops with their
parent chain and input shapes.

    python tools/probes/dropin_ops_probe.py
"""
from __future__ import annotations

import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bbgr  # noqa: E402,F401
from bbgr import lightgcn_cu_pop as V2  # noqa: E402
from bbgr.optim import FusedAdam  # noqa: E402
from bbgr.synthetic import synthetic_credibility, synthetic_edges  # noqa: E402


def main():
    U, I, E, d, K, B = 200_000, 50_000, 2_000_000, 64, 3, 8192
    dev = "cuda"
    e = synthetic_edges(U, I, E, seed=1, items="zipf")
    cred = torch.as_tensor(synthetic_credibility(U, 2))
    M_ui, M_iu = V2.build_message_passing_mats(e, U, I, cred, dev)
    m = V2.LightGCN(U, I, d, K, M_ui, M_iu).to(dev)
    opt = FusedAdam(m.parameters(), lr=1e-3)
    g = torch.Generator(device=dev).manual_seed(0)

    def step():
        users = torch.randint(0, U, (B,), device=dev, generator=g)
        pos = torch.randint(0, I, (B,), device=dev, generator=g)
        neg = torch.randint(0, I, (B,), device=dev, generator=g)
        uf, itf = m.propagate()
        loss = m.bpr_loss(users, pos, neg, uf, itf, 1e-4)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    keep = ("copy", "clone", "contiguous", "to_dense", "coalesce", "add", "mul", "index",
            "zeros", "fill", "cat", "sort", "cummax", "where", "arange")
    for ev in prof.events():
        if ev.device_type != torch.autograd.DeviceType.CPU or not ev.name.startswith("aten::"):
            continue
        if not any(k in ev.name for k in keep):
            continue
        chain, p = [], ev.cpu_parent
        while p is not None and len(chain) < 4:
            chain.append(p.name)
            p = p.cpu_parent
        print(f"{ev.name:34s} {str(ev.input_shapes)[:60]:60s} <- {' <- '.join(chain)[:150]}")
    print(prof.key_averages().table(sort_by="device_time_total", row_limit=25))


if __name__ == "__main__":
    main()
