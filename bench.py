"""Benchmark: LightGCN propagation + BPR training step on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C4]

A "step" is one full training step of Version-2/lighgcn_cu_pop.py:826-866 on
one batch: pop-mix sampling -> K-layer GS propagation (2K fused SpMMs) ->
fused BPR -> backward (2K transposed SpMMs) -> Adam on every parameter.
Inputs (graph, operators, tables) are resident in HBM before timing starts.

value = SpMM edges/s of the whole job = 4*K*E edges traversed per step
        * steps / wall time (max over ranks). BPR steps/s is reported beside.
roofline = the fused SpMM kernel (dominant kernel): algorithmic bytes per launch
        B = E*(4 + 4 + 4d) + R*(4 + 4d) / average launch time,
        measured with events around every SpMM launch inside the timed region.
cpu_baseline = the reference's CPU path (oracle/ref_torch.py: the same torch
        calls) timed on this host on a bounded sample (see "sample").
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# More hardware queues than HIP's default 4, so the compute stream, RCCL's stream
# and the sharded exchange's side streams do not share (and serialise on) one
# AQL queue. Must be set before the HIP runtime initialises.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import bbgr  # noqa: E402,F401
from bbgr import propagate as P  # noqa: E402
from bbgr.synthetic import (CONFIGS, CONFIG_SEED, config_edges, shard_edges_strong,  # noqa: E402
                            shard_edges_weak, synthetic_credibility)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic():
    """Per-launch HBM bytes of spmm_kernel from the latest committed rocprofv3
    PMC passes (tools/profile_box.sh + tools/summarize_profile.py)."""
    p = os.path.join(ROOT, "profiles", "spmm_traffic.json")
    if not os.path.exists(p):
        return None, None
    j = json.load(open(p))
    return j.get("hbm_bytes_per_launch_corrected"), j.get("source")


def spmm_bytes(nnz: int, rows: int, d: int) -> int:
    return nnz * (4 + 4 + 4 * d) + rows * (4 + 4 * d)


def spmm_adam_bytes(nnz: int, rows: int, d: int) -> int:
    """Last backward product with the user Adam in its epilogue: the SpMM bytes
    minus the gradient write, plus param / exp_avg / exp_avg_sq read + write."""
    return spmm_bytes(nnz, rows, d) - rows * 4 * d + 6 * rows * 4 * d


def cpu_baseline(edges, cfg, batch, sample_users=256):
    """Reference CPU path (same torch calls) on a bounded sample of the step."""
    from oracle import ref_numpy as R
    from oracle import ref_torch as T
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    cores = max(1, min(cores, os.cpu_count() or 1))
    torch.set_num_threads(cores)
    U, I, d, K = cfg["num_users"], cfg["num_items"], cfg["emb_dim"], cfg["num_layers"]
    E = edges.shape[1]
    M_ui, M_iu = T.gs_operators(edges, U, I)            # not timed (operator build)
    g = torch.Generator().manual_seed(0)
    u0 = torch.rand(U, d, generator=g) - 0.5
    i0 = torch.rand(I, d, generator=g) - 0.5
    t0 = time.perf_counter()
    torch.sparse.mm(M_iu, u0)
    t_iu = time.perf_counter() - t0
    t0 = time.perf_counter()
    torch.sparse.mm(M_ui, i0)
    t_ui = time.perf_counter() - t0
    del M_ui, M_iu
    # Adam over every parameter (dense, as the reference's dense grads force)
    pu = torch.nn.Parameter(u0)
    pi = torch.nn.Parameter(i0)
    opt = torch.optim.Adam([pu, pi], lr=1e-3)
    pu.grad, pi.grad = torch.zeros_like(u0), torch.zeros_like(i0)
    t0 = time.perf_counter()
    opt.step()
    t_adam = time.perf_counter() - t0
    # the reference's per-user pop-mix sampler loop on a user subset
    indptr, indices = R.edges_to_user_csr(edges, U)
    pp = R.pop_prob(edges, I)
    rng = np.random.default_rng(42)
    users = rng.choice(np.flatnonzero(np.diff(indptr) > 0), sample_users, replace=False)
    t0 = time.perf_counter()
    R.sample_batch_reference_style(indptr, indices, users, I, rng, pp)
    t_samp = (time.perf_counter() - t0) * batch / sample_users
    t_step = K * (t_iu + t_ui) * 2 + t_adam + t_samp
    return {
        "value": 4 * K * E / t_step, "unit": "edges/s", "cores": cores, "kind": "port",
        "sample": (f"{cfg_name_global}: one torch.sparse.mm per direction "
                   f"(item<-user {t_iu:.2f}s, user<-item {t_ui:.2f}s) x2K for fwd+bwd, "
                   f"torch Adam on all {U + I} rows ({t_adam:.2f}s), reference pop-mix "
                   f"sampler loop on {sample_users} users scaled to B={batch} "
                   f"({t_samp:.2f}s); est. {t_step:.1f}s/step"),
        "step_s": t_step,
    }


cfg_name_global = "C4"


def _quiet_stdout():
    """Route fd 1 to stderr (collective libraries print banners on stdout) and
    return a writer for the real stdout: the JSON line is its only content."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(saved, "w")


def main():
    global cfg_name_global
    out_stream = _quiet_stdout()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C4")
    ap.add_argument("--variant", default="v2_pop")
    ap.add_argument("--cred", default="beta", choices=["beta", "ones"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dense", action="store_true",
                    help="disable exact frontier sparsity (every SpMM over the full CSR)")
    ap.add_argument("--sharded", action="store_true",
                    help="run the multi-GPU trainer (torch.distributed) even at N=1: "
                         "measures the sharded step's own overhead, collectives included")
    ap.add_argument("--exchange-parts", type=int, default=8,
                    help="N>1: item-row ranges per dense exchange (all-reduce of range c "
                         "overlaps the SpMM of range c+1)")
    ap.add_argument("--vertex-order", default="degree", choices=["degree", "input"],
                    help="number users / items by descending degree inside the graph "
                         "(hot rows cached, cold rows streamed) or keep the input ids")
    ap.add_argument("--native-comm", action="store_true",
                    help="N>1: item all-reduces through the C ABI's own RCCL communicator "
                         "(bbgr_allreduce_items) instead of torch.distributed")
    ap.add_argument("--frontier-parts", type=int, default=2,
                    help="N>1: item-row ranges per frontier (row-list) exchange")
    ap.add_argument("--dense-check", type=int, default=5,
                    help="after the timed steps, time this many steps with frontier sparsity "
                         "off (reported as dense_ms_per_step; 0 = skip)")
    ap.add_argument("--roofline-steps", type=int, default=3,
                    help="sharded runs: steps after the timed region whose SpMM launches "
                         "are bracketed by HIP events for the roofline")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="N>1: weak = every rank owns a full config-sized user shard over the "
                         "shared items; strong = one config graph cut into N user ranges")
    args = ap.parse_args()
    cfg_name_global = args.config
    cfg = CONFIGS[args.config]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    local = local % max(torch.cuda.device_count(), 1)   # ranks may share a GPU (gloo rehearsal)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist_mode = world > 1 or args.sharded
    if dist_mode:
        # RCCL ("nccl") in production; BBGR_DIST_BACKEND=gloo lets two ranks
        # share one GPU to rehearse the multi-rank path on a 1-GPU box.
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29577")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        backend = os.environ.get("BBGR_DIST_BACKEND", "nccl")
        if backend == "nccl":
            # high-priority RCCL stream: its kernels get CUs while the SpMM of the
            # next item range floods the queue (range_probe: 2.07 -> 1.96 ms / product)
            opts = torch.distributed.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
            torch.distributed.init_process_group("nccl", device_id=dev, pg_options=opts)
        else:
            torch.distributed.init_process_group(backend)

    U, I, d, K = cfg["num_users"], cfg["num_items"], cfg["emb_dim"], cfg["num_layers"]
    B = cfg["batch"]
    weak = world > 1 and args.scaling == "weak"
    # configs too large to draw whole on every rank (C5) are drawn per user shard
    sharded_gen = not weak and cfg["num_edges"] > 100_000_000
    t0 = time.perf_counter()
    seed = CONFIG_SEED[args.config]
    lo = hi = 0
    if weak:
        edges = shard_edges_weak(args.config, rank)
        cred = synthetic_credibility(U, seed + 7919 * rank, args.cred)
        E = edges.shape[1] * world                       # edges of the whole job's graph
    elif sharded_gen:
        edges, lo, hi = shard_edges_strong(args.config, rank, world)
        cred = synthetic_credibility(hi - lo, seed + 7919 * rank, args.cred)
        E = cfg["num_edges"]
    else:
        edges = config_edges(args.config)
        cred = synthetic_credibility(U, seed, args.cred)
        E = edges.shape[1]
    log(f"[bench] rank {rank}: {args.config} U={U} I={I} E={E} d={d} K={K} B={B} "
        f"scaling={args.scaling} generated in {time.perf_counter() - t0:.1f}s")

    xp = dict(exchange_parts=args.exchange_parts, frontier_parts=args.frontier_parts,
              vertex_order=args.vertex_order)
    if args.native_comm:
        xp["native_comm"] = True
    if not dist_mode:
        from bbgr.graph import BipartiteGraph
        from bbgr.trainer import FusedTrainer
        graph = BipartiteGraph(edges, U, I, dev, vertex_order=args.vertex_order)
        trainer = FusedTrainer(graph, args.variant, cred=cred, emb_dim=d, num_layers=K,
                               batch_size=B, frontier=not args.dense)
    elif weak:
        from bbgr.distributed import ShardedTrainer
        trainer = ShardedTrainer(edges, U, I, args.variant, cred=cred, emb_dim=d,
                                 num_layers=K, batch_size=B, device=dev, user_offset=rank * U,
                                 frontier=not args.dense, **xp)
    elif sharded_gen:
        from bbgr.distributed import ShardedTrainer
        trainer = ShardedTrainer(edges, hi - lo, I, args.variant, cred=cred, emb_dim=d,
                                 num_layers=K, batch_size=max(1, B // world), device=dev,
                                 user_offset=lo, frontier=not args.dense, **xp)
    else:
        from bbgr.distributed import ShardedTrainer
        trainer = ShardedTrainer.from_global_edges(edges, U, I, args.variant, cred=cred,
                                                   emb_dim=d, num_layers=K, batch_size=B,
                                                   device=dev, frontier=not args.dense, **xp)
    if dist_mode:
        del edges   # the cpu_baseline leg (rank 0, N=1 only) is the only later user
    torch.cuda.synchronize()
    log(f"[bench] rank {rank}: setup done, {torch.cuda.memory_allocated(dev) / 2**30:.1f} GiB")

    for _ in range(args.warmup):
        trainer.step()
    timer = P.SpmmTimer()
    if dist_mode:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    # Per-launch HIP events for the roofline. On one GPU they ride inside the
    # timed steps (cost ~0.1 ms/step). In the sharded step, events recorded
    # between launches interleave with the collectives' cross-stream waits and
    # cost 1.4-3 ms/step (15-step runs at N=1: 19.4-21.1 ms with them, 18.0-18.1
    # without), so
    # there the events are recorded over `--roofline-steps` extra steps right
    # after the timed region instead.
    events_in_loop = not dist_mode
    if events_in_loop:
        P.set_spmm_timer(timer)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = trainer.step()
    torch.cuda.synchronize()
    if dist_mode:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    P.set_spmm_timer(None)
    timer_steps = args.steps
    if not events_in_loop:
        timer_steps = max(1, args.roofline_steps)
        P.set_spmm_timer(timer)
        for _ in range(timer_steps):
            trainer.step()
        torch.cuda.synchronize()
        P.set_spmm_timer(None)
    if dist_mode:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss)
    dense_ms = None
    if not args.dense and args.dense_check > 0:
        # the same trainer with frontier sparsity off (every product over the
        # full CSR): what the masks save, reported next to the value
        trainer.frontier = False
        trainer.step()
        if dist_mode:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.dense_check):
            trainer.step()
        torch.cuda.synchronize()
        if dist_mode:
            torch.distributed.barrier()
        dense_s = time.perf_counter() - t1
        if dist_mode:
            t = torch.tensor([dense_s], device=dev, dtype=torch.float64)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            dense_s = float(t.item())
        dense_ms = 1000.0 * dense_s / args.dense_check
        trainer.frontier = True
    if dist_mode:
        trainer.close()                    # the native exchange's communicator, if any
    summ = timer.summary("full")          # full-CSR launches: the roofline kernel
    summ_m = timer.summary("masked")       # frontier-masked launches (bytes data-dependent)
    summ_a = timer.summary("adam")         # last backward product + fused user Adam
    tot_bytes = sum(n * spmm_bytes(nnz, rows, dd) for (rows, nnz, dd), (n, ms) in summ.items())
    tot_ms = sum(ms for (n, ms) in summ.values())
    n_launch = sum(n for (n, ms) in summ.values())
    per_kernel = {f"rows{rows}_nnz{nnz}_d{dd}": {"launches": n, "avg_ms": ms / n,
                                                 "GBps": n * spmm_bytes(nnz, rows, dd) / (ms * 1e6)}
                  for (rows, nnz, dd), (n, ms) in summ.items()}
    achieved = tot_bytes / (tot_ms * 1e6) if tot_ms > 0 else 0.0   # GB/s
    masked_ms = sum(ms for (n, ms) in summ_m.values())
    masked_n = sum(n for (n, ms) in summ_m.values())
    adam_info = {f"rows{rows}_nnz{nnz}_d{dd}": {
        "launches": n, "avg_ms": ms / n,
        "algorithmic_bytes": spmm_adam_bytes(nnz, rows, dd),
        "GBps": n * spmm_adam_bytes(nnz, rows, dd) / (ms * 1e6)}
        for (rows, nnz, dd), (n, ms) in summ_a.items()}
    traffic, traffic_src = pmc_traffic() if (args.config == "C4" and world == 1) else (None, None)
    edges_per_step = 4 * K * E
    if rank != 0:
        if dist_mode:
            torch.distributed.destroy_process_group()
        return
    cpu = None
    if not args.no_cpu_baseline and not dist_mode and not sharded_gen:
        log("[bench] timing the reference CPU path (bounded sample) ...")
        cpu = cpu_baseline(edges, cfg, B)
    out = {
        "metric": "SpMM edges/sec + BPR steps/sec, |E|=50M d=64, 1/2/4/8 MI355X; %HBM roofline",
        "value": edges_per_step * args.steps / elapsed,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1000.0 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": args.scaling,   # N=1: weak and strong are the same run
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (Zipf-0.8 items, geometric user degrees; xavier init; Beta cred)",
        "config": {"workload": f"{args.config} BPR training step ({args.variant})"
                               + (f", {world} x {args.config} user shards" if weak else ""),
                   "num_users": U * (world if weak else 1), "num_items": I, "num_edges": E,
                   "vertex_order": args.vertex_order,
                   "emb_dim": d, "num_layers": K,
                   "global_batch": B * (world if weak else 1),
                   "parallelism": f"user-rows x{world}"
                                  + (" (sharded trainer)" if dist_mode and world == 1 else "")},
        "bpr_steps_per_s": args.steps / elapsed,
        "dense_ms_per_step": dense_ms,
        "dense_note": "same trainer, frontier sparsity off (every SpMM over the full CSR; "
                      "loss, gradients and updates equal): timed after the main loop",
        "spmm_edges_per_s_kernel": (E * n_launch) / (tot_ms / 1e3) if tot_ms else None,
        "frontier": {"enabled": not args.dense,
                     "masked_launches_per_step": masked_n / timer_steps,
                     "masked_ms_per_step": masked_ms / timer_steps,
                     "full_launches_per_step": n_launch / timer_steps,
                     "full_sequence_ms": [
                         {"rows": r, "nnz": z, "avg_ms": ms}
                         for r, z, ms in timer.sequence("full", timer_steps)],
                     "adam_sequence_ms": [
                         {"rows": r, "nnz": z, "avg_ms": ms}
                         for r, z, ms in timer.sequence("adam", timer_steps)],
                     "masked_sequence_ms": [
                         {"rows": r, "nnz": z, "avg_ms": ms}
                         for r, z, ms in timer.sequence("masked", timer_steps)],
                     "note": "value counts the reference step's 4*K*E edge traversals; "
                             "masked launches skip exact-zero / unread rows"},
        "fused_adam_spmm": adam_info,
        "final_loss": final_loss,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_unit": "bytes/launch (2*FETCH_SIZE+WRITE_SIZE, rocprofv3)",
                     "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": tot_bytes / max(n_launch, 1),
                     "kernel": "bbgr::spmm_kernel / spmm_pair_kernel (+fixup)", "launches": n_launch,
                     "avg_launch_ms": tot_ms / max(n_launch, 1), "per_operator": per_kernel,
                     "events": "inside the timed steps" if events_in_loop else
                               f"{timer_steps} steps after the timed region (sharded step)",
                     "cache_assisted": achieved > HBM_PEAK_GBS,
                     "note": "achieved = gather-model bytes (zero reuse) / launch time; above "
                             "peak only because hot rows are served from L2 / Infinity Cache "
                             "(degree order + streamed cold rows); `traffic` is the PMC-measured "
                             "HBM bytes per launch"},
        "cpu_baseline": None if cpu is None else {k: v for k, v in cpu.items() if k != "step_s"},
    }
    print(json.dumps(out), file=out_stream, flush=True)
    if dist_mode:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
