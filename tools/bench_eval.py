"""Benchmark: sampled evaluation on MI355X.

    python tools/bench_eval.py [--config C4] [--reps 5] [--cpu-users 40000] [--full]

Workload: the C4 synthetic graph (5M users x 1M items, 50M interactions);
20% of the interactions (seeded) are held out as the test split, the rest is
the train split. Embeddings are random (metric values are irrelevant to the
timing; the protocol is: every user with a test item gets 1 pos + 99 negatives
rejected against its test and train rows, K = 10, 20).

value = evaluated users / wall time of one bbgr.evaluation.evaluate_sampled
        call (inputs resident in HBM; includes the host read-back of the sums).
roofline = eval_sampled_kernel: algorithmic bytes per user = (1 + n_neg + 1)
        rows of d fp32 (the user row and every candidate's item row) / launch
        time, timed with HIP events on the launching stream.
--stream numpy: the candidates of the reference's own numpy stream
        (np.random.default_rng(seed + 999), drawn on the host by
        bbgr_eval_draw_candidates, bit for bit the reference loop's), uploaded
        and scored by the same kernel; the host draw is timed apart
        (host_draw_s) and included in the wall time.
--full: the full-ranking protocol; roofline = fp32 MFMA (2*d flops per
        (user, item) score) over the whole evaluate_full device time.
cpu_baseline = the reference's per-user loop restated in oracle/ref_numpy.py
        (evaluate_sampled_reference_style, numpy RNG + searchsorted rejection +
        per-user scoring and metrics) on a bounded sample of users.
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
from bbgr.evaluation import evaluate_full, evaluate_sampled  # noqa: E402
from bbgr.graph import Csr  # noqa: E402
from bbgr.synthetic import CONFIGS, config_edges, synthetic_credibility  # noqa: E402

HBM_PEAK_GBS = 8000.0
FP32_MFMA_PEAK_TF = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def split(edges, frac, seed):
    rng = np.random.default_rng([seed, 0x7E57])
    test = rng.random(edges.shape[1]) < frac
    return np.ascontiguousarray(edges[:, ~test]), np.ascontiguousarray(edges[:, test])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--negatives", type=int, default=99)
    ap.add_argument("--cpu-users", type=int, default=40000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ks", type=int, nargs="+", default=[10, 20],
                    help="--full: the cutoffs (the top-K list is max(ks) deep)")
    ap.add_argument("--full", action="store_true",
                    help="full-ranking protocol (evaluate_full_ranking) instead of sampled")
    ap.add_argument("--stream", default="philox", choices=["philox", "numpy"],
                    help="sampled: device Philox candidates, or the reference's numpy stream")
    ap.add_argument("--max-users", type=int, default=0,
                    help="evaluate only the first N users with test items (0 = all)")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    U, I, d = cfg["num_users"], cfg["num_items"], cfg["emb_dim"]
    dev = "cuda"
    t0 = time.perf_counter()
    edges = config_edges(args.config)
    tr, te = split(edges, 0.2, 5)
    del edges
    log(f"[eval] {args.config}: train {tr.shape[1]} test {te.shape[1]} ({time.perf_counter()-t0:.1f}s)")
    trc = Csr(tr[0], tr[1], U, I, dev)
    tec = Csr(te[0], te[1], U, I, dev)
    g = torch.Generator(device=dev).manual_seed(7)
    uf = (torch.rand(U, d, device=dev, generator=g) - 0.5)
    itf = (torch.rand(I, d, device=dev, generator=g) - 0.5)
    pop = np.bincount(tr[1], minlength=I).astype(np.float32)
    pop_t = torch.tensor(pop, device=dev)
    cred = synthetic_credibility(U, 3)
    cred_t = torch.tensor(cred, device=dev, dtype=torch.float32)
    T = int(tr.shape[1])
    if args.max_users:   # restrict the test split to the first N users that have test items
        keep_u = np.unique(te[0])[: args.max_users]
        te = te[:, np.isin(te[0], keep_u)]
        tec = Csr(te[0], te[1], U, I, dev)
    if args.full:
        run = lambda c: evaluate_full(uf, itf, trc, tec, I, pop_t, T, cred_t,  # noqa: E731
                                      Ks=tuple(args.ks))
    elif args.stream == "numpy":
        from bbgr import evaluation as EV
        from bbgr.host_sampler import edges_to_user_csr
        tr_csr, te_csr = edges_to_user_csr(tr, U), edges_to_user_csr(te, U)
        host_users = np.where(np.diff(te_csr[0]) > 0)[0].astype(np.int64)
        users_t = torch.from_numpy(host_users).to(dev)
        groups_t = torch.from_numpy(EV.cred_group_flags(host_users, cred, 0.2)).to(dev)
        draw_s = []

        def run(c):
            t = time.perf_counter()
            cand = EV.draw_candidates(np.random.default_rng(42 + 999), host_users, tr_csr,
                                      te_csr, I, args.negatives)
            draw_s.append(time.perf_counter() - t)
            return evaluate_sampled(uf, itf, trc, tec, I, pop_t, T, cred_t,
                                    sampled_negatives=args.negatives,
                                    cand=torch.from_numpy(cand).pin_memory(), users=users_t,
                                    groups=groups_t)
    else:
        run = lambda c: evaluate_sampled(uf, itf, trc, tec, I, pop_t, T, cred_t,  # noqa: E731
                                         sampled_negatives=args.negatives, counter=c)
    for w in range(args.warmup):
        run(w)
    torch.cuda.synchronize()
    # kernel time: HIP events on the launching stream around the whole call
    s = torch.cuda.current_stream()
    evs = []
    walls = []
    res = None
    for r in range(args.reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        a.record(s)
        res = run(100 + r)
        b.record(s)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t1)
        evs.append(a.elapsed_time(b) / 1e3)
    k0 = args.ks[0] if args.full else 10
    n_eval = int(res[k0]["users_eval"])
    wall = float(np.median(walls))
    dev_s = float(np.median(evs))
    nc = 1 + args.negatives
    if args.full:   # MFMA-bound: 2*d flops per (user, item) score
        alg = 2.0 * n_eval * I * d
        roof = {"bound": "mfma", "achieved": alg / dev_s / 1e12, "peak": FP32_MFMA_PEAK_TF,
                "unit": "TFLOP/s", "frac": alg / dev_s / 1e12 / FP32_MFMA_PEAK_TF,
                "traffic": None, "note": "whole evaluate_full device time (score+top-K, merge, "
                                         "metrics); fp32 MFMA dense peak"}
    else:
        alg = n_eval * (nc + 1) * d * 4
        roof = {"bound": "hbm", "achieved": alg / dev_s / 1e9, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": alg / dev_s / 1e9 / HBM_PEAK_GBS, "traffic": None,
                "note": "whole evaluate_sampled device time (sample+score+rank, metrics)"}
    log(f"[eval] users {n_eval}  wall {wall*1e3:.2f} ms  device {dev_s*1e3:.2f} ms  "
        f"ndcg@{k0} {res[k0]['ndcg']:.4f}")
    cpu = None
    if not args.no_cpu_baseline:
        from oracle import ref_numpy as R
        trp, tri = R.edges_to_user_csr(tr, U)
        tep, tei = R.edges_to_user_csr(te, U)
        n_cpu = max(1, args.cpu_users // 400) if args.full else args.cpu_users
        users = np.where(np.diff(tep) > 0)[0][:n_cpu]
        ufn, itn = uf.cpu().numpy(), itf.cpu().numpy()
        t1 = time.perf_counter()
        if args.full:
            ranked = R.full_ranking_reference_style(users, trp, tri, ufn, itn, 20)
            hi, lo = R.make_cred_groups(users, cred, 0.2)
            R.evaluate_given_topk(users, ranked, tep, tei, pop, T, I, cred, hi, lo)
        else:
            R.evaluate_sampled_reference_style(trp, tri, tep, tei, ufn, itn, I, pop, T, cred,
                                               n_neg=args.negatives, users=users)
        el = time.perf_counter() - t1
        cpu = {"value": users.size / el, "unit": "users/s", "cores": 1, "kind": "port",
               "sample": f"reference per-user loop (oracle restatement) on the first "
                         f"{users.size} evaluated users of the same split: {el:.1f} s"}
        log(f"[eval] cpu {users.size} users {el:.1f}s -> {users.size/el:.0f} users/s")
    kstr = ",".join(str(k) for k in args.ks)
    proto = f"full ranking (all items, K={kstr})" if args.full else \
        f"sampled eval (1 pos + {args.negatives} neg, K=10,20; {args.stream} candidates)"
    line = {
        "metric": "eval_users_per_s", "value": n_eval / wall, "unit": "users/s",
        "n_gpus": 1, "steps": args.reps, "warmup": args.warmup, "ms_per_step": wall * 1e3,
        "higher_is_better": True, "scaling": "none", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": f"{args.config} {proto}",
                   "users_eval": n_eval, "num_items": I, "emb_dim": d,
                   "train_edges": T, "test_edges": int(te.shape[1])},
        "device_ms": dev_s * 1e3,
        "host_draw_s": (float(np.median(draw_s)) if not args.full and args.stream == "numpy"
                        else None),
        "candidate_stream": None if args.full else args.stream,
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
