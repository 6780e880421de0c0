"""Benchmark: credibility-GNN aggregation on MI355X.

    python tools/bench_cred.py [--config C4] [--reps 5] [--hidden 64]

Workload: the C4 synthetic interaction graph as the user->item edge set
(5M users, 1M items, 50M edges) with random 5-column edge attributes
(EDGE_ATTR_KEYS), hidden width 64. One pass = what CredModel.forward_subgraph
(main.py:693-707) does to the edges, plus the aggregation backward of a
training step: EWA weights + per-destination normalisation for both
directions, aggregate users->items, aggregate items->users, and the two
transposed products of the backward. The CSRs are built once (a graph).

value = edges/s = 4 * E / pass time (four weighted aggregations per pass).
roofline = the aggregation SpMM (spmm_kernel, explicit edge values):
        algorithmic bytes E*(4 + 4 + 4d) + R*(4 + 4d) per launch / launch time.
cpu_baseline = the reference formulation (oracle/ref_torch.CredModelRef's
        ewa_raw / normalize_per_dst / aggregate: index_add_ scatters) on this
        host's cores over a bounded edge sample, scaled to E.
Prints ONE JSON line on stdout.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bbgr  # noqa: E402,F401
from bbgr import propagate as P  # noqa: E402
from bbgr.cred_gnn import EdgeSet, aggregate  # noqa: E402
from bbgr.synthetic import CONFIGS, config_edges  # noqa: E402

HBM_PEAK_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--hidden", type=int, default=64)
    ap.add_argument("--cpu-edges", type=int, default=2_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    U, I, d = cfg["num_users"], cfg["num_items"], args.hidden
    dev = "cuda"
    edges = config_edges(args.config)
    E = edges.shape[1]
    rng = np.random.default_rng(0)
    ea = rng.uniform(-0.2, 1.2, (E, 5)).astype(np.float32)
    t0 = time.perf_counter()
    e_t = torch.from_numpy(edges.astype(np.int64)).to(dev)
    s1 = EdgeSet(e_t, U, I)                        # users -> items
    s2 = EdgeSet(torch.stack([e_t[1], e_t[0]]), I, U)   # items -> users
    ea_t = torch.from_numpy(ea).to(dev)
    torch.cuda.synchronize()
    log(f"[cred] {args.config}: E={E} edge sets built in {time.perf_counter() - t0:.1f}s")
    h_u = torch.randn(U, d, device=dev) * 0.1
    h_i = torch.randn(I, d, device=dev) * 0.1
    g_i = torch.randn(I, d, device=dev) * 0.1
    g_u = torch.randn(U, d, device=dev) * 0.1

    def one_pass():
        _, w1, w1c = s1.normalize(edge_attr=ea_t)
        _, w2, w2c = s2.normalize(edge_attr=ea_t)
        xu = h_u.requires_grad_(True)
        xi = h_i.requires_grad_(True)
        m_i = aggregate(xu, s1, w1, w1c)
        m_u = aggregate(xi, s2, w2, w2c)
        torch.autograd.backward([m_i, m_u], [g_i, g_u])
        xu.grad = None
        xi.grad = None

    for _ in range(args.warmup):
        one_pass()
    torch.cuda.synchronize()
    timer = P.SpmmTimer()
    P.set_spmm_timer(timer)
    t0 = time.perf_counter()
    for _ in range(args.reps):
        one_pass()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / args.reps
    P.set_spmm_timer(None)
    summ = timer.summary("full")
    tot_b = sum(n * (nnz * (8 + 4 * dd) + rows * (4 + 4 * dd)) for (rows, nnz, dd), (n, ms) in summ.items())
    tot_ms = sum(ms for n, ms in summ.values())
    n_l = sum(n for n, ms in summ.values())
    ach = tot_b / (tot_ms * 1e6)
    log(f"[cred] pass {el * 1e3:.2f} ms; aggregation SpMM {tot_ms / n_l:.3f} ms avg, {ach:.0f} GB/s")
    cpu = None
    if not args.no_cpu_baseline:
        from oracle.ref_torch import CredModelRef
        n = min(args.cpu_edges, E)
        cores = max(1, min(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)),
                           os.cpu_count() or 1))
        torch.set_num_threads(cores)
        m = CredModelRef(1, 1, d)
        ei = torch.from_numpy(edges[:, :n].astype(np.int64))
        eat = torch.from_numpy(ea[:n])
        xu = (torch.randn(U, d) * 0.1).requires_grad_(True)
        xi = (torch.randn(I, d) * 0.1).requires_grad_(True)
        t1 = time.perf_counter()
        w1 = m.normalize_per_dst(m.ewa_raw(eat), ei[1], I)
        w2 = m.normalize_per_dst(m.ewa_raw(eat), ei[0], U)
        m_i = m.aggregate(xu, ei, w1, I)
        m_u = m.aggregate(xi, torch.stack([ei[1], ei[0]]), w2, U)
        torch.autograd.backward([m_i, m_u], [torch.ones_like(m_i), torch.ones_like(m_u)])
        c_el = time.perf_counter() - t1
        cpu = {"value": 4 * n / c_el, "unit": "edges/s", "cores": cores, "kind": "port",
               "sample": f"reference index_add_ formulation (CredModelRef) on the first {n} "
                         f"edges, fwd + bwd of both aggregations: {c_el:.2f} s"}
        log(f"[cred] cpu {n} edges {c_el:.2f}s")
    line = {
        "metric": "cred_gnn_aggregation_edges_per_s", "value": 4 * E / el, "unit": "edges/s",
        "n_gpus": 1, "steps": args.reps, "warmup": args.warmup, "ms_per_step": el * 1e3,
        "higher_is_better": True, "scaling": "none", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (C4 graph, uniform edge attributes)",
        "config": {"workload": f"{args.config} cred-GNN EWA weights + 2 aggregations fwd+bwd",
                   "num_users": U, "num_items": I, "num_edges": E, "hidden": d},
        "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": ach / HBM_PEAK_GBS, "traffic": None,
                     "kernel": "bbgr::spmm_kernel (explicit edge values)", "launches": n_l,
                     "avg_launch_ms": tot_ms / n_l},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
