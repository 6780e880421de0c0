"""Cache-reuse probe: item-row SpMM (gathers from the user table) at fixed
E = 50M, I = 1M Zipf items, d = 64, for user tables of decreasing size.
Algorithmic TB/s well above the HBM peak at small tables = L2/MALL serving
the gathers (the premise of column-blocked propagation)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bbgr  # noqa: E402,F401
from bbgr.graph import Csr  # noqa: E402
from bbgr.propagate import Product, spmm  # noqa: E402
from bbgr.synthetic import _zipf_sampler  # noqa: E402

E, I, d = 50_000_000, 1_000_000, 64
rng = np.random.default_rng(0)
draw = _zipf_sampler(I, 0.8, rng, 4)
items = draw(E).astype(np.int32)
for U in [int(a) for a in (sys.argv[1:] or ["5000000", "2000000", "1000000", "500000", "250000", "125000"])]:
    users = rng.integers(0, U, E).astype(np.int32)
    c = Csr(items, users, I, U, "cuda")
    prod = Product(c, None, None, None, {})
    x = torch.randn(U, d, device="cuda")
    y = torch.empty(I, d, device="cuda")
    for _ in range(2):
        spmm(prod, x, False, y=y)
    torch.cuda.synchronize()
    n = 5
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        spmm(prod, x, False, y=y)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    alg = E * (4 + 4 * d) + I * (4 + 4 * d)
    print(f"U={U:>8d} table={U * d * 4 / 2**20:7.1f} MiB  {ms:.3f} ms  alg {alg / ms / 1e9:.2f} TB/s",
          flush=True)
    del c, prod, x
