"""Probe: cost of autograd's dense += sparse-COO accumulation on the GPU
(how the drop-in's sparse ego-L2 rows reach .grad), uncoalesced vs marked
coalesced, at the C4 table sizes, with the kernels each launches.

    python tools/probes/sparse_add_probe.py
"""
import torch
from torch.profiler import ProfilerActivity, profile


def run(rows, n, coalesced):
    dev = "cuda"
    dense = torch.randn(rows, 64, device=dev)
    idx = torch.randint(0, rows, (n,), device=dev)
    if coalesced:
        idx = torch.unique(idx)
    vals = torch.randn(idx.numel(), 64, device=dev)
    if coalesced:
        sp = torch.sparse_coo_tensor(idx.unsqueeze(0), vals, (rows, 64), is_coalesced=True)
    else:
        sp = torch.sparse_coo_tensor(idx.unsqueeze(0), vals, (rows, 64))
    for _ in range(3):
        dense.add_(sp)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        dense.add_(sp)
    e1.record()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        dense.add_(sp)
        torch.cuda.synchronize()
    ks = [(e.key[:60], round(e.device_time_total, 1)) for e in prof.key_averages() if e.device_time_total > 0]
    print(rows, n, "coalesced" if coalesced else "uncoalesced",
          round(e0.elapsed_time(e1) / 10 * 1e3, 1), "us", ks, flush=True)


for rows, n in ((1_000_000, 16384), (5_000_000, 8192)):
    for c in (False, True):
        run(rows, n, c)
