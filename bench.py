"""Benchmark: LightGCN propagation + BPR training step on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C4]

A "step" is one full training step of Version-2/lighgcn_cu_pop.py:826-866 on
one batch: pop-mix sampling -> K-layer GS propagation (2K fused SpMMs) ->
fused BPR -> backward (2K transposed SpMMs) -> Adam on every parameter.
Inputs (graph, operators, tables) are resident in HBM before timing starts.

value = SpMM edges actually gathered per second, whole job: every launch's
        gathered edges (source row read and multiply-added; frontier-masked
        launches count only their live edges) counted on the device over
        --count-steps steps after the timed region, x steps / wall time of the
        timed steps (max over ranks). BPR steps/s and the reference-equivalent
        4*K*E edges per step are reported beside it.
roofline = the dominant kernel (full-CSR item<-user spmm_kernel): gather-model
        bytes per launch B = E*(4 + 4 + 4d) + R*(4 + 4d) / its
        average launch time from HIP events on the launching stream (inside the
        timed steps on one GPU; over --roofline-steps eager steps after them for
        sharded / graph-replayed runs). `cache_assisted` flags a gather-model
        rate above the guide's measured ceiling for random whole-row gathers
        from HBM (5.8 TB/s): such a rate is served partly by L2 / the Infinity
        Cache. Step level: the PMC bytes of one whole step (profiles/
        step_traffic.json, rocprofv3 2*FETCH_SIZE+WRITE_SIZE summed over the
        step's kernels) / ms_per_step, beside the summed gather-model bytes.
cpu_baseline = the reference's CPU path (oracle/ref_torch.py: the same torch
        calls) timed on this host on a bounded sample (see "sample").
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time

# More hardware queues than HIP's default 4, so the compute stream, RCCL's stream
# and the sharded exchange's side streams do not share (and serialise on) one
# AQL queue. Must be set before the HIP runtime initialises.
HW_QUEUES_GIVEN = os.environ.get("GPU_MAX_HW_QUEUES")
if int(HW_QUEUES_GIVEN or 0) < 8 and os.environ.get("BBGR_KEEP_HW_QUEUES") != "1":
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import bbgr  # noqa: E402,F401
from bbgr import _lib  # noqa: E402
from bbgr import propagate as P  # noqa: E402
from bbgr.synthetic import (CONFIGS, CONFIG_SEED, config_edges, shard_edges_strong,  # noqa: E402
                            shard_edges_weak, synthetic_credibility)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec
# MI355X_MICROARCH.md (Infinity Cache section): random whole rows of a buffer far
# larger than the Infinity Cache, each fetched once, read at 5.5-5.8 TB/s
# chip-wide (6.3 TB/s for an in-order stream). A gather-model rate above this is
# cache-assisted: part of the modelled bytes come from L2 / the Infinity Cache.
HBM_GATHER_CEILING_GBS = 5800.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def spmm_bytes(nnz: int, rows: int, d: int) -> int:
    return nnz * (4 + 4 + 4 * d) + rows * (4 + 4 * d)


def spmm_adam_bytes(nnz: int, rows: int, d: int) -> int:
    """Last backward product with the user Adam in its epilogue: the SpMM bytes
    minus the gradient write, plus param / exp_avg / exp_avg_sq read + write."""
    return spmm_bytes(nnz, rows, d) - rows * 4 * d + 6 * rows * 4 * d


def spmm_adam_side_bytes(nnz: int, rows: int, d: int) -> int:
    """A product that still writes its output and carries another table's Adam
    (the GS item Adam on the last backward item product): the SpMM bytes plus
    the gradient row read and param / exp_avg / exp_avg_sq read + write."""
    return spmm_bytes(nnz, rows, d) + 7 * rows * 4 * d


def _median_s(fn, reps: int = 5, warmup: int = 1):
    """Median wall time of fn() over `reps` runs after `warmup` untimed runs.
    fn may return its own measured seconds (a sub-interval); else the call is timed."""
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        ts.append(r if isinstance(r, float) else time.perf_counter() - t0)
    return float(np.median(ts)), ts


def _spread(ts) -> dict:
    """Run-to-run spread of a list of timings: interquartile range and full
    range, each relative to the median."""
    q25, q50, q75 = np.percentile(ts, [25, 50, 75])
    return {"iqr_rel": float((q75 - q25) / q50), "range_rel": float((max(ts) - min(ts)) / q50)}


def _reference_step_s(cfg_name: str, variant: str = "v2_pop", reps: int = 11):
    """Median seconds of one whole reference-style training step at a small
    config, the variant's own family (oracle/ref_torch.reference_model):
    the per-user sampler loop (pop-mix: Version-2/lighgcn_cu_pop.py:835-849;
    uniform: lightgcn_cu.py:611-621 / lightgcn.py:565-575), then propagate ->
    bpr_loss -> backward -> Adam (V2:858-863, cu:632-652, lightgcn.py:584-589)."""
    from oracle import ref_numpy as R
    from oracle import ref_torch as T
    c = CONFIGS[cfg_name]
    U, I, d, K, B = c["num_users"], c["num_items"], c["emb_dim"], c["num_layers"], c["batch"]
    e = config_edges(cfg_name)
    cred = synthetic_credibility(U, CONFIG_SEED[cfg_name])
    torch.manual_seed(42)
    model, popmix = T.reference_model(variant, e, U, I, d, K, cred)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    indptr, indices = R.edges_to_user_csr(e, U)
    pp = R.pop_prob(e, I)
    rng = np.random.default_rng(42)
    train_users = np.flatnonzero(np.diff(indptr) > 0)
    perm = rng.permutation(train_users)
    pos_in_perm = [0]

    def step():
        lo = pos_in_perm[0] % max(len(perm) - B, 1)
        pos_in_perm[0] += B
        users = perm[lo:lo + B]
        if popmix:
            us, ps, ns = R.sample_batch_reference_style(indptr, indices, users, I, rng, pp)
        else:
            us, ps, ns = R.sample_batch_uniform_reference_style(indptr, indices, users, I, rng)
        T.train_step(model, opt, torch.as_tensor(us), torch.as_tensor(ps),
                     torch.as_tensor(ns), 1e-4)

    med, ts = _median_s(step, reps)
    return med, ts, 4 * K * e.shape[1]


def _cpu_list_text(cpus) -> str:
    """[0,1,2,3,8] -> "0-3,8"."""
    cpus = sorted(cpus)
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


def cpu_threads() -> int:
    """Threads for the CPU baseline: every CPU this process may run on (its
    affinity set; BASELINE.md §2: torch.set_num_threads(os.cpu_count())),
    capped by the host's CPU share for this job when the environment states
    one (OMP_NUM_THREADS: the GPU box sets it to its per-GPU share, 16, while
    os.cpu_count() and the affinity set show the whole shared machine)."""
    n = max(1, len(os.sched_getaffinity(0)))
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return n


def cpu_baseline(edges, cfg, cfg_name, cred, variant: str = "v2_pop",
                 whole_steps=("C2", "C1"), whole_reps: int = 11,
                 small_edges: int = 4_000_000, seed: int = 42):
    """The reference's CPU path (oracle/ref_torch.py: the same torch calls as
    Version-2/lighgcn_cu_pop.py:441-450, 482-489, 858-863, lightgcn_cu.py:
    420-448, 632-652, lightgcn.py:318-349) timed on this host with every CPU
    of the process's affinity set, for the bench's variant.

    C1 / C2 (small graphs): whole reference steps end to end (sampler loop,
    propagate, loss, backward, Adam), median of `whole_reps` after one warm-up,
    with the run-to-run spread.

    C3 / C4 (50M edges): ONE whole reference training step, measured: the
    variant's per-user sampler loop over the full batch of B users
    (Version-2:835-849), then loss = bpr(propagate()) (2K torch.sparse.mm over
    every edge), loss.backward() (autograd's 2K transposed products) and
    torch.optim.Adam.step() over all (U+I) x d parameters (V2:858-863), each
    part timed. One run (a step takes minutes of host time); the whole
    reference steps of the same variant at C2 and C1 are timed FIRST, so
    torch's CPU thread pool, sparse kernels and allocator are warm when the C4
    step starts (its large tensors are fresh mmaps in every step of the
    reference too, so their first-touch cost belongs to the step)."""
    from oracle import ref_numpy as R
    from oracle import ref_torch as T
    cores = cpu_threads()
    torch.set_num_threads(cores)
    U, I, d, K, B = (cfg["num_users"], cfg["num_items"], cfg["emb_dim"], cfg["num_layers"],
                     cfg["batch"])
    E = edges.shape[1]
    if E <= small_edges:   # C1 / C2: the whole step, end to end
        med, ts, work = _reference_step_s(cfg_name, variant, whole_reps)
        return {"value": work / med, "unit": "edges/s", "cores": cores, "kind": "port",
                "bpr_steps_per_s": 1.0 / med, "step_s": med,
                "sample": (f"whole {cfg_name} reference steps ({variant}: sampler loop, "
                           f"propagate, BPR, backward, Adam), median of {whole_reps} after "
                           f"1 warm-up: {med:.3f}s"),
                "whole_step_s": {cfg_name: {"median": med, "runs": ts, "edges_per_s": work / med,
                                            **_spread(ts)}}}
    whole = {n: _reference_step_s(n, variant, whole_reps) for n in whole_steps}
    t_setup = time.perf_counter()
    torch.manual_seed(seed)
    model, popmix = T.reference_model(variant, edges, U, I, d, K, cred)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    indptr, indices = R.edges_to_user_csr(edges, U)
    pp = R.pop_prob(edges, I) if popmix else None
    rng = np.random.default_rng(seed)
    users = rng.permutation(np.flatnonzero(np.diff(indptr) > 0))[:B]
    t_setup = time.perf_counter() - t_setup
    # the variant's per-user sampler loop over the whole batch (single thread)
    t0 = time.perf_counter()
    if popmix:
        us, ps, ns = R.sample_batch_reference_style(indptr, indices, users, I, rng, pp)
    else:
        us, ps, ns = R.sample_batch_uniform_reference_style(indptr, indices, users, I, rng)
    t_samp = time.perf_counter() - t0
    del indptr, indices
    us, ps, ns = (torch.as_tensor(x) for x in (us, ps, ns))
    # propagate + BPR loss, backward, Adam: T.train_step split at its parts
    t0 = time.perf_counter()
    loss = model.loss(us, ps, ns, 1e-4)
    t1 = time.perf_counter()
    opt.zero_grad()
    loss.backward()
    t2 = time.perf_counter()
    opt.step()
    t3 = time.perf_counter()
    loss_v = float(loss.item())
    del loss, opt, model
    t_fwd, t_bwd, t_adam = t1 - t0, t2 - t1, t3 - t2
    t_step = t_samp + t_fwd + t_bwd + t_adam
    return {
        "value": 4 * K * E / t_step, "unit": "edges/s", "cores": cores, "kind": "port",
        "bpr_steps_per_s": 1.0 / t_step,
        "sample": (f"ONE whole {cfg_name} {variant} reference step, measured (one run, after "
                   f"the C2 / C1 whole steps warmed torch's CPU machinery): "
                   f"{'pop-mix' if popmix else 'uniform'} sampler loop over B={B} "
                   f"users {t_samp:.1f}s (1 thread), propagate + BPR {t_fwd:.1f}s (2K={2 * K} "
                   f"torch.sparse.mm over all {E} edges), loss.backward() {t_bwd:.1f}s, torch "
                   f"Adam over {U + I} rows {t_adam:.2f}s: {t_step:.1f}s/step on {cores} "
                   f"threads. Whole reference steps, median of {whole_reps}: "
                   + ", ".join(f"{n} {w[0]:.3f}s ({w[2] / w[0] / 1e6:.1f} M edges/s)"
                               for n, w in whole.items())),
        "step_s": t_step,
        "step_measured": True,
        "loss": loss_v,
        "components_s": {"sampler": t_samp, "forward_bpr": t_fwd, "backward": t_bwd,
                         "adam": t_adam},
        "whole_step_s": {n: {"median": w[0], "runs": w[1], "edges_per_s": w[2] / w[0],
                             **_spread(w[1])} for n, w in whole.items()},
        "setup_s": t_setup,
        "os_cpu_count": os.cpu_count(),
        "affinity_cpus": len(os.sched_getaffinity(0)),
        "threads_note": "threads = the affinity set, capped by the job's CPU share "
                        "(OMP_NUM_THREADS on the GPU box: 16 per GPU of a shared host)",
    }


cfg_name_global = "C4"


def _quiet_stdout():
    """Route fd 1 to stderr (collective libraries print banners on stdout) and
    return a writer for the real stdout: the JSON line is its only content."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(saved, "w")


def _allreduce(x: float, dev, op) -> float:
    t = torch.tensor([x], device=dev, dtype=torch.float64)
    torch.distributed.all_reduce(t, op=op)
    return float(t.item())


def edges_per_step(counts: dict, d: int, steps: int) -> tuple[float, float]:
    """(gathered, visited) edges per step from SpmmTimer.edge_counts(). A
    launch over a column slice (column shards, column chains) gathers
    d_launch / d of each edge's row and counts as that fraction of an edge."""
    gathered = sum(c[3] * k[4] / d for k, c in counts.items()) / steps
    visited = sum(c[2] * k[4] / d for k, c in counts.items()) / steps
    return gathered, visited


def _compulsory_bytes(nnz: int, rows: int, n_cols: int, d: int) -> int:
    """every edge's index + weight once, every source row
    once, every output row (+ indptr) once: E*8 + C*4d + R*(4 + 4d)."""
    return nnz * 8 + n_cols * 4 * d + rows * (4 + 4 * d)


def roofline_groups(timer, counts, steps: int, count_steps: int, n_items: int):
    """Per launch kind and side: launches, average ms, gather-model and
    compulsory-model bytes per launch, their GB/s and fractions of 8 TB/s.
    Full-CSR / range launches take their bytes from the CSR; masked launches
    from the rows / edges counted on the device over `count_steps` extra steps."""
    out = []
    for (kind, sig, tr, nc, d), (n, ms, rows, nnz) in sorted(timer.groups().items()):
        side = "item<-user" if tr == n_items else "user<-item"
        e = {"kind": kind, "side": side, "d": d, "launches_per_step": n / steps,
             "avg_ms": ms / n}
        if kind == "masked":
            e["masks"] = sig
            c = counts.get((kind, sig, tr, nc, d))
            if not c:
                continue
            cn, crows, cvis, cgat = c
            rows_l, vis_l, gat_l = crows / cn, cvis / cn, cgat / cn
            e["rows_per_launch"], e["edges_visited_per_launch"] = rows_l, vis_l
            e["edges_gathered_per_launch"] = gat_l
            gather = vis_l * 8 + gat_l * 4 * d + rows_l * (4 + 4 * d)
            compulsory = None
        else:
            rows_l, nnz_l = rows / n, nnz / n
            gather = (spmm_bytes if kind == "full" else spmm_adam_side_bytes
                      if kind == "adam_side" else spmm_adam_bytes)(nnz_l, rows_l, d)
            compulsory = _compulsory_bytes(nnz_l, rows_l, nc, d) + \
                {"full": 0, "adam": 5, "adam_side": 7}[kind] * rows_l * 4 * d
            e["rows_per_launch"], e["edges_per_launch"] = rows_l, nnz_l
        e["gather_model_bytes"] = gather
        e["gather_model_GBps"] = gather / (e["avg_ms"] * 1e6)
        e["gather_model_frac"] = e["gather_model_GBps"] / HBM_PEAK_GBS
        e["cache_assisted"] = e["gather_model_GBps"] > HBM_GATHER_CEILING_GBS
        if compulsory is not None:
            e["compulsory_bytes"] = compulsory
            e["compulsory_GBps"] = compulsory / (e["avg_ms"] * 1e6)
            e["compulsory_frac"] = e["compulsory_GBps"] / HBM_PEAK_GBS
        out.append(e)
    return out


def step_traffic():
    """PMC bytes of one whole C4 training step (profiles/step_traffic.json,
    tools/summarize_profile.py over a tools/profile_box.sh run)."""
    p = os.path.join(ROOT, "profiles", "step_traffic.json")
    if not os.path.exists(p):
        return None
    return json.load(open(p))


def pmc_traffic():
    """Per-launch HBM bytes of the dominant kernel (item<-user spmm_kernel) from
    the committed rocprofv3 PMC passes (tools/profile_box.sh +
    tools/summarize_profile.py), with the commit and tag they were taken at."""
    p = os.path.join(ROOT, "profiles", "spmm_traffic.json")
    if not os.path.exists(p):
        return None
    return json.load(open(p))


def measure_weak(args, cfg, rank: int, world: int, dev, xp: dict, frontier) -> dict:
    """`--weak-beside` steps of the weak-scaled sharded step (N x the config's
    edges, N x its batch): timed like the main loop (barrier + sync on both
    sides, max over ranks), gathered edges counted over one extra step."""
    from bbgr.distributed import ShardedTrainer
    U, I, d, K, B = (cfg["num_users"], cfg["num_items"], cfg["emb_dim"], cfg["num_layers"],
                     cfg["batch"])
    seed = CONFIG_SEED[args.config]
    edges = shard_edges_weak(args.config, rank)
    cred = synthetic_credibility(U, seed + 7919 * rank, args.cred)
    # full config-sized shards: the item products hide the exchange themselves
    # (range pipeline); column chains would only add compute
    xpw = dict(xp, column_chains=1, exchange_parts=4, frontier_parts=2)
    tr = ShardedTrainer(edges, U, I, args.variant, cred=cred, emb_dim=d, num_layers=K,
                        batch_size=B, device=dev, user_offset=rank * U, frontier=frontier,
                        **xpw)
    E = int(_allreduce(tr.graph.item_csr.nnz, dev, torch.distributed.ReduceOp.SUM))
    del edges
    for _ in range(max(1, args.warmup)):
        tr.step()
    torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.weak_beside):
        tr.step()
    torch.cuda.synchronize()
    torch.distributed.barrier()
    el = _allreduce(time.perf_counter() - t0, dev, torch.distributed.ReduceOp.MAX)
    counter = P.SpmmTimer(count=True)
    P.set_spmm_timer(counter)
    tr.step()
    torch.cuda.synchronize()
    P.set_spmm_timer(None)
    gathered = _allreduce(edges_per_step(counter.edge_counts(), d, 1)[0],
                          dev, torch.distributed.ReduceOp.SUM)
    tr.close()
    steps_per_s = args.weak_beside / el
    return {"value": gathered * steps_per_s, "unit": "edges/s", "scaling": "weak",
            "ms_per_step": 1000.0 * el / args.weak_beside, "steps": args.weak_beside,
            "bpr_steps_per_s": steps_per_s, "num_edges": E, "num_users": U * world,
            "global_batch": tr.B_global,
            "note": f"{world} x {args.config} user shards over the shared items, measured "
                    "after the strong line in the same run"}


# --graph auto: replay the step as one HIP graph below this many edges (C1,
# C2: launch-bound steps; at C4 replay and eager tie)
GRAPH_MAX_EDGES = 4_000_000

# per-rank compute of the C4 user-row step at N = 8, measured alone (DESIGN
# §6: one chain with inline collectives / two column chains): the constants of
# the chain-setting rule; other (config, N) have no measured constants
RANK_COMPUTE_MS = {("C4", 8): {"inline": 2.39, "two_chains": 2.90}}


def allreduce_probe(dev, world: int, native: bool, sizes, iters: int = 5) -> dict:
    """The item exchange's all-reduce alone: `sizes` bytes of fp32 through
    torch's process group and (RCCL only) the C ABI's communicator inline on
    the current stream, each timed over `iters` calls between a barrier + sync
    on both sides, max over ranks. t_ar per call; bus bandwidth = 2(P-1)/P x
    bytes / t_ar (a ring all-reduce's per-rank wire bytes), algorithm
    bandwidth = bytes / t_ar."""
    from bbgr.distributed import RcclItemComm
    out = {"world": world, "iters": iters, "sizes_bytes": list(sizes)}
    comm, err = None, None
    if native:   # a communicator that will not come up costs the C ABI figures only
        try:
            comm = RcclItemComm(device=dev, inline=True)
        except Exception as ex:   # noqa: BLE001
            err = f"{type(ex).__name__}: {ex}"[:300]
        if _allreduce(0.0 if comm is None else 1.0, dev, torch.distributed.ReduceOp.MIN) < 1.0:
            out["cabi_error"] = err or "the C ABI communicator failed on another rank"
            if comm is not None:
                comm.close()
            comm = None
    try:
        for S in sizes:
            t = torch.ones(S // 4, dtype=torch.float32, device=dev)
            ways = [("torch", lambda: torch.distributed.all_reduce(t))]
            if comm is not None:
                ways.append(("cabi", lambda: comm.all_reduce(t)))
            for name, run in ways:
                for _ in range(2):
                    run()
                torch.cuda.synchronize()
                torch.distributed.barrier()
                t0 = time.perf_counter()
                for _ in range(iters):
                    run()
                torch.cuda.synchronize()
                torch.distributed.barrier()
                el = _allreduce(time.perf_counter() - t0, dev, torch.distributed.ReduceOp.MAX)
                t_ar = el / iters
                out[f"{name}_{S >> 20}MB"] = {
                    "t_ar_ms": 1e3 * t_ar,
                    "busbw_GBps": 2.0 * (world - 1) / world * S / t_ar / 1e9,
                    "algbw_GBps": S / t_ar / 1e9}
            del t
    finally:
        if comm is not None:
            comm.close()
    return out


def chain_rule(probe: dict, config: str, world: int, K: int, dense_bytes: int,
               frontier_bytes: int) -> dict | None:
    """DESIGN §6 / §8 item 1 on the measured t_ar: one inline chain takes
    n_dense t_ar(dense) + n_frontier t_ar(frontier) + its compute; two column
    chains overlap the exchange with the other chain's products,
    max(exchange, compute). The predicted faster setting runs first; both
    are timed and the measured faster is the line."""
    c = RANK_COMPUTE_MS.get((config, world))
    if c is None or probe is None:
        return None
    key = lambda how, S: probe.get(f"{how}_{S >> 20}MB", {}).get("t_ar_ms")  # noqa: E731
    n_dense, n_front = 2 * (K - 1), 2
    inline_how = "cabi" if key("cabi", dense_bytes) is not None else "torch"
    wire_inline = n_dense * key(inline_how, dense_bytes) + n_front * key(inline_how, frontier_bytes)
    wire_two = n_dense * key("torch", dense_bytes) + n_front * key("torch", frontier_bytes)
    pred_inline = wire_inline + c["inline"]
    pred_two = max(wire_two, c["two_chains"])
    return {"exchanges_per_step": {"dense": n_dense, "frontier": n_front},
            "rank_compute_ms": c, "wire_ms": {"inline": wire_inline, "two_chains": wire_two},
            "predicted_ms": {"inline": pred_inline, "two_chains": pred_two},
            "predicted": "inline" if pred_inline < pred_two else "two_chains"}


def step_summary(ms, dense_ms, torch_ref, dropin, dropin_fused, dropin_bwd) -> dict:
    """The step times of the line and of the runs beside it, in one small
    object printed last (the driver keeps the tail of stdout)."""
    def ms_of(r):
        return None if r is None else round(r["step_ms"], 3)
    return {"ms_per_step": round(ms, 3),
            "dense_ms_per_step": None if not dense_ms else round(dense_ms, 3),
            "torch_gpu_reference_step_ms": ms_of(torch_ref),
            "dropin_module_step_ms": ms_of(dropin),
            "dropin_fused_adam_step_ms": ms_of(dropin_fused),
            "dropin_backward_adam_step_ms": ms_of(dropin_bwd),
            "note": "ms per step: the fused trainer (the line), its dense form, the reference's "
                    "step in stock PyTorch-ROCm, the drop-in module with torch's foreach Adam / "
                    "FusedAdam / FusedAdam(fuse_backward=True)"}


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
    ap.add_argument("--no-torch-reference", action="store_true",
                    help="skip timing the reference step in stock PyTorch on the GPU")
    ap.add_argument("--dense", action="store_true",
                    help="disable exact frontier sparsity (every SpMM over the full CSR)")
    ap.add_argument("--frontier", default="auto", choices=["auto", "on", "off"],
                    help="frontier masks: auto = the trainer's size rule")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="single GPU: replay the step as one captured HIP graph "
                         "(trainer.GraphedStep); auto = on below the frontier size rule's "
                         "edge count (launch-bound small graphs)")
    ap.add_argument("--sharded", action="store_true",
                    help="run the multi-GPU trainer (torch.distributed) even at N=1: "
                         "measures the sharded step's own overhead, collectives included")
    ap.add_argument("--exchange-parts", type=int, default=None,
                    help="N>1: item-row ranges per dense exchange (all-reduce of range c "
                         "overlaps the SpMM of range c+1). Each range costs a launch tail "
                         "and a collective call: one C4 rank of 8 measured 3.10 / 3.18 / "
                         "3.43 / 4.00 ms of compute with 1 / 2 / 4 / 8 ranges "
                         "(tools/shard_probe.py), against ≤ t_item*(1-1/P) of hidden wire "
                         "time per exchange. Default 1 with column chains (the other chain "
                         "hides the wire time), else 4")
    ap.add_argument("--vertex-order", default="degree", choices=["degree", "input"],
                    help="number users / items by descending degree inside the graph "
                         "(hot rows cached, cold rows streamed) or keep the input ids")
    ap.add_argument("--native-comm", nargs="?", const="stream", default="off",
                    choices=["off", "stream", "inline"],
                    help="N>1 user rows: the item exchange through the C ABI's own RCCL "
                         "communicator (bbgr_allreduce_items) on a comm stream ('stream', "
                         "the bare flag), or every collective of the step inline on the "
                         "compute stream ('inline': one column chain)")
    ap.add_argument("--column-chains", type=int, default=None,
                    help="users partition: run the propagation as this many column chains "
                         "(d/C columns each, own stream, issue interleaved per exchange) so "
                         "one chain's SpMMs overlap another's item all-reduces. Default: 2 "
                         "for strong scaling at N >= 8 with <= 20M edges per rank (one C4 rank "
                         "of 8 computes in 3.38 ms with 2 chains and no ranges, as with 1 "
                         "chain and 4 ranges), else 1")
    ap.add_argument("--frontier-parts", type=int, default=None,
                    help="N>1: item-row ranges per frontier (row-list) exchange")
    ap.add_argument("--dense-check", type=int, default=5,
                    help="after the timed steps, time this many steps with frontier sparsity "
                         "off (reported as dense_ms_per_step; 0 = skip)")
    ap.add_argument("--count-steps", type=int, default=3,
                    help="steps after the timed region whose launches count the rows / edges "
                         "they actually process (value = traversed edges)")
    ap.add_argument("--roofline-steps", type=int, default=3,
                    help="sharded runs: steps after the timed region whose SpMM launches "
                         "are bracketed by HIP events for the roofline")
    ap.add_argument("--partition", default="auto", choices=["auto", "columns", "users"],
                    help="N>1 strong scaling: columns = every rank the whole graph and d/N "
                         "embedding columns (no item exchange; 12 B per triple all-reduced); "
                         "users = user-row shards with item all-reduces (DESIGN §6); auto = "
                         "columns when d/N is a supported width and the graph is drawn whole")
    ap.add_argument("--emulate-columns", type=int, default=0,
                    help="single GPU: run ONE column shard of N (d/N columns, the whole graph) "
                         "alone, the per-rank work of a column-sharded N-GPU step")
    ap.add_argument("--weak-beside", type=int, default=10,
                    help="N>1 strong runs: afterwards time this many weak-scaled steps "
                         "(each rank a full config-sized shard) and report them beside "
                         "the strong line (0 = skip)")
    ap.add_argument("--ar-probe", type=int, default=1,
                    help="N > 1: time the item all-reduce alone first (allreduce_probe)")
    ap.add_argument("--dist-timeout", type=float, default=180.0,
                    help="N>1: seconds before a stuck collective aborts the run (every rank "
                         "draws its graph in parallel first: C4 ~25 s)")
    ap.add_argument("--partition-beside", type=int, default=1,
                    help="strong N > 1: also time the other partition (columns / users) on "
                         "the same graph and report the faster as the line (0 = off)")
    ap.add_argument("--chain-beside", type=int, default=1,
                    help="strong N > 1, user-row partition: also time the step as ONE chain "
                         "with no item-row ranges and every collective inline on the compute "
                         "stream (the C ABI's RCCL communicator; over gloo, where RCCL cannot "
                         "share a GPU, the same one-chain schedule through torch's "
                         "collectives) beside the default chain setting; the faster is the "
                         "line, the other is reported as chain_beside (0 = off)")
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"],
                    help="N>1: strong (default) = the config's one graph cut into N user "
                         "ranges (the metric's |E|); weak = every rank owns a full "
                         "config-sized user shard over the shared items")
    args = ap.parse_args()
    cfg_name_global = args.config
    cfg = CONFIGS[args.config]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    scaling = args.scaling or "strong"
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
        # a collective stuck on one rank aborts the job after --dist-timeout
        # seconds (torch's watchdog names the op, its sequence number and size)
        # instead of sitting until the driver kills the run
        timeout = datetime.timedelta(seconds=args.dist_timeout)
        if backend == "nccl":
            # high-priority RCCL stream: its kernels get CUs while the SpMM of the
            # next item range floods the queue (range_probe: 2.07 -> 1.96 ms / product)
            opts = torch.distributed.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
            torch.distributed.init_process_group("nccl", device_id=dev, pg_options=opts,
                                                 timeout=timeout)
        else:
            torch.distributed.init_process_group(backend, timeout=timeout)

    U, I, d, K = cfg["num_users"], cfg["num_items"], cfg["emb_dim"], cfg["num_layers"]
    B = cfg["batch"]
    weak = world > 1 and scaling == "weak"
    # configs too large to draw whole on every rank (C5) are drawn per user shard
    sharded_gen = not weak and cfg["num_edges"] > 100_000_000
    from bbgr.columns import MIN_AUTO_WIDTH, can_shard_columns
    partition = args.partition
    if partition == "auto":
        # columns while the shards stay >= 16 columns wide (C4: N = 2, 4),
        # user rows beyond
        partition = ("columns" if world > 1 and not weak and not sharded_gen
                     and can_shard_columns(d, world, MIN_AUTO_WIDTH) else "users")
    columns = dist_mode and partition == "columns" and not weak
    if columns:
        sharded_gen = False
    emulate = args.emulate_columns if not dist_mode else 0
    t0 = time.perf_counter()
    seed = CONFIG_SEED[args.config]
    lo = hi = 0
    if weak:
        edges = shard_edges_weak(args.config, rank)
        cred = synthetic_credibility(U, seed + 7919 * rank, args.cred)
    elif sharded_gen:
        edges, lo, hi = shard_edges_strong(args.config, rank, world)
        cred = synthetic_credibility(hi - lo, seed + 7919 * rank, args.cred)
    else:
        edges = config_edges(args.config)
        cred = synthetic_credibility(U, seed, args.cred)
    log(f"[bench] rank {rank}: {args.config} U={U} I={I} d={d} K={K} B={B} "
        f"scaling={scaling} generated in {time.perf_counter() - t0:.1f}s")

    # the item all-reduce alone (dense payload I*d*4, frontier 16 MB) before any
    # step: t_ar and bus bandwidth on this machine's links (DESIGN §6 assumed
    # 76.8 GB/s per link)
    ar_probe = None
    if world > 1 and args.ar_probe:
        ar_probe = allreduce_probe(dev, world, backend == "nccl", (I * d * 4, 16 << 20))
        log(f"[bench] rank {rank}: all-reduce probe {json.dumps(ar_probe)}")
    rule = chain_rule(ar_probe, args.config, world, K, I * d * 4, 16 << 20) \
        if (args.column_chains is None and args.native_comm == "off" and not weak) else None
    if args.native_comm == "inline":   # one chain, no ranges: nothing overlaps the wire
        args.column_chains = 1
        args.exchange_parts = 1 if args.exchange_parts is None else args.exchange_parts
        args.frontier_parts = 1 if args.frontier_parts is None else args.frontier_parts
    if args.column_chains is None:
        # small per-rank shards only: there the exchange outlasts the rank's
        # item products; a big shard's item product hides it by itself (C5)
        small = cfg["num_edges"] // max(world, 1) <= 20_000_000
        args.column_chains = 2 if (world >= 8 and not weak and small and d % 2 == 0
                                   and d // 2 in (8, 16, 32, 64, 128)) else 1
    if args.exchange_parts is None:
        args.exchange_parts = 1 if args.column_chains > 1 else 4
    if args.frontier_parts is None:   # with chains the other chain hides the wire time
        args.frontier_parts = 1 if args.column_chains > 1 else 2
    xp = dict(exchange_parts=args.exchange_parts, frontier_parts=args.frontier_parts,
              vertex_order=args.vertex_order)
    if args.native_comm != "off":
        xp["native_comm"] = True if args.native_comm == "stream" else "inline"
    if args.column_chains > 1:
        xp["column_chains"] = args.column_chains
    frontier = {"auto": "auto", "on": True, "off": False}[args.frontier]
    if args.dense:
        frontier = False
    def build(part: str, xpo: dict | None = None):
        """The trainer of one partition ("columns" / "users" at N > 1); xpo:
        the user-row exchange settings (default: xp)."""
        xq = xp if xpo is None else xpo
        if emulate:
            from bbgr.columns import ColumnShardedTrainer
            return ColumnShardedTrainer(edges, U, I, args.variant, cred=cred, emb_dim=d,
                                        num_layers=K, batch_size=B, device=dev,
                                        vertex_order=args.vertex_order, frontier=frontier,
                                        column_parts=emulate, column_index=0)
        if not dist_mode:
            from bbgr.graph import BipartiteGraph
            from bbgr.trainer import FusedTrainer
            graph = BipartiteGraph(edges, U, I, dev, vertex_order=args.vertex_order)
            return FusedTrainer(graph, args.variant, cred=cred, emb_dim=d, num_layers=K,
                                batch_size=B, frontier=frontier)
        if part == "columns":
            from bbgr.columns import ColumnShardedTrainer
            return ColumnShardedTrainer(edges, U, I, args.variant, cred=cred, emb_dim=d,
                                        num_layers=K, batch_size=B, device=dev,
                                        vertex_order=args.vertex_order, frontier=frontier)
        from bbgr.distributed import ShardedTrainer
        if weak:
            return ShardedTrainer(edges, U, I, args.variant, cred=cred, emb_dim=d,
                                  num_layers=K, batch_size=B, device=dev, user_offset=rank * U,
                                  frontier=frontier, **xq)
        if sharded_gen:
            return ShardedTrainer(edges, hi - lo, I, args.variant, cred=cred, emb_dim=d,
                                  num_layers=K, batch_size=max(1, B // world), device=dev,
                                  user_offset=lo, frontier=frontier, **xq)
        return ShardedTrainer.from_global_edges(edges, U, I, args.variant, cred=cred,
                                                emb_dim=d, num_layers=K, batch_size=B,
                                                device=dev, frontier=frontier, **xq)

    count_steps = max(1, args.count_steps)

    def measure(trainer, part: str, dense_check: int) -> dict:
        """Warm-up, then EXACTLY args.steps timed steps (barrier + sync on both
        sides, max over ranks); per-launch events, device edge counts and the
        dense (frontier off) step after the timed region."""
        cols = dist_mode and part == "columns"
        # edges of the whole job's graph: the sum of the ranks' shards (column
        # shards all hold the whole graph)
        E_local = trainer.graph.item_csr.nnz
        E = int(_allreduce(E_local, dev, torch.distributed.ReduceOp.SUM)) if dist_mode and \
            not cols else E_local
        torch.cuda.synchronize()
        log(f"[bench] rank {rank}: {part} setup done, E={E} (local {E_local}), frontier="
            f"{trainer.frontier}, {torch.cuda.memory_allocated(dev) / 2**30:.1f} GiB")
        use_graph = not dist_mode and (args.graph == "on" or (args.graph == "auto"
                                                              and E < GRAPH_MAX_EDGES))
        step_fn = trainer.step
        if use_graph:
            from bbgr.trainer import GraphedStep
            step_fn = GraphedStep(trainer).step
        for _ in range(args.warmup):
            step_fn()
        timer = P.SpmmTimer()
        # in the timed steps only the dominant launches (full-CSR item<-user
        # products) carry events: an event pair costs ~10 us of idle GPU around
        # its launch (r6b timeline: 12 timed launches, ~0.12 ms per step); the
        # other kinds are timed over --roofline-steps eager steps afterwards
        n_items_local = trainer.graph.item_csr.n_rows
        dom_timer = P.SpmmTimer(select=lambda kind, prod: kind == "full"
                                and prod.csr.n_rows == n_items_local)
        if dist_mode:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        # Per-launch HIP events for the roofline. On one GPU they ride inside the
        # timed steps (cost ~0.1 ms/step). In the sharded step, events recorded
        # between launches interleave with the collectives' cross-stream waits and
        # cost 1.4-3 ms/step, so there the events are recorded over
        # `--roofline-steps` extra steps right after the timed region instead.
        # A captured graph replays its launches without the host: its per-launch
        # events are taken over eager steps after the timed region, as for sharded.
        events_in_loop = not dist_mode and not use_graph
        if events_in_loop:
            P.set_spmm_timer(dom_timer)
        # rocprofv3 runs (tools/profile_box.sh) cut the trace at two empty marker
        # kernels around the timed steps: per-step dispatch counts are exact
        marks = os.environ.get("BBGR_PROFILE_MARKS") == "1"
        if marks:
            _lib.call("bbgr_profile_marker", 1, _lib.stream_handle())
        t0 = time.perf_counter()
        for _ in range(args.steps):
            loss = step_fn()
        if marks:
            _lib.call("bbgr_profile_marker", 2, _lib.stream_handle())
        torch.cuda.synchronize()
        if dist_mode:
            torch.distributed.barrier()
        elapsed = time.perf_counter() - t0
        P.set_spmm_timer(None)
        timer_steps = max(1, args.roofline_steps)
        P.set_spmm_timer(timer)
        for _ in range(timer_steps):
            trainer.step()
        torch.cuda.synchronize()
        P.set_spmm_timer(None)
        if dist_mode:
            elapsed = _allreduce(elapsed, dev, torch.distributed.ReduceOp.MAX)
        final_loss = float(loss)
        # rows / edges every launch actually processes (frontier masks make them
        # data-dependent), counted on the device over extra steps
        counter = P.SpmmTimer(count=True)
        P.set_spmm_timer(counter)
        for _ in range(count_steps):
            trainer.step()
        torch.cuda.synchronize()
        P.set_spmm_timer(None)
        counts = counter.edge_counts()
        gathered_step, visited_step = edges_per_step(counts, d, count_steps)
        if dist_mode:
            gathered_step = _allreduce(gathered_step, dev, torch.distributed.ReduceOp.SUM)
            visited_step = _allreduce(visited_step, dev, torch.distributed.ReduceOp.SUM)
        dense_ms = None
        if trainer.frontier and dense_check > 0:
            # the same trainer with frontier sparsity off (every product over the
            # full CSR): what the masks save, reported next to the value
            trainer.frontier = False
            trainer.step()
            if dist_mode:
                torch.distributed.barrier()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(dense_check):
                trainer.step()
            torch.cuda.synchronize()
            if dist_mode:
                torch.distributed.barrier()
            dense_s = time.perf_counter() - t1
            if dist_mode:
                dense_s = _allreduce(dense_s, dev, torch.distributed.ReduceOp.MAX)
            dense_ms = 1000.0 * dense_s / dense_check
            trainer.frontier = True
        return dict(part=part, columns=cols, E=E, use_graph=use_graph, timer=timer,
                    dom_timer=dom_timer if events_in_loop else None,
                    timer_steps=timer_steps, events_in_loop=events_in_loop, elapsed=elapsed,
                    final_loss=final_loss, counts=counts, gathered_step=gathered_step,
                    visited_step=visited_step, dense_ms=dense_ms,
                    frontier_on=bool(trainer.frontier),
                    value=gathered_step * args.steps / elapsed,
                    ms_per_step=1000.0 * elapsed / args.steps)

    backend_nccl = dist_mode and torch.distributed.get_backend() == "nccl"
    # the user-row step as ONE chain with every collective in issue order on
    # the compute stream: through the C ABI's RCCL communicator,
    # or over gloo (ranks sharing a GPU, where RCCL cannot run) the same
    # one-chain, one-range schedule through torch's collectives
    inline_xp = None
    if args.native_comm != "inline":
        inline_xp = dict(xp, exchange_parts=1, frontier_parts=1)
        inline_xp.pop("column_chains", None)
        inline_xp.pop("native_comm", None)
        if backend_nccl:
            inline_xp["native_comm"] = "inline"

    def chain_mode(xq: dict) -> str:
        nc = xq.get("native_comm")
        c = xq.get("column_chains", 1)
        if nc == "inline":
            return "1 chain, every collective inline on the compute stream (C ABI RCCL)"
        how = ("C ABI RCCL on a comm stream" if nc else "torch collectives")
        return f"{c} chain{'s' if c > 1 else ''}, {xq['exchange_parts']} item-row range(s), {how}"

    if ar_probe is not None and ar_probe.get("cabi_error") and inline_xp is not None:
        # the C ABI communicator did not come up on this machine: the one-chain
        # setting runs its collectives through torch's group instead
        inline_xp.pop("native_comm", None)
    # the user-row chain settings: the main run and the one beside it (the
    # probe's rule, when it has constants, decides which runs first)
    main_xp, beside_xp = xp, inline_xp
    if rule is not None and rule["predicted"] == "inline" and inline_xp is not None:
        main_xp, beside_xp = inline_xp, xp
    U_job = U * (world if weak else 1)
    strong_multi = dist_mode and world > 1 and not weak
    todo = [(partition, main_xp if partition == "users" else xp)]
    if strong_multi and partition == "users" and args.chain_beside and beside_xp is not None:
        todo.append(("users", beside_xp))
    other = {"columns": "users", "users": "columns"}.get(partition)
    if (strong_multi and not sharded_gen and args.partition_beside
            and (other == "users" or can_shard_columns(d, world))):
        # strong N > 1: the other partition, measured the same way right after;
        # the faster one is the line, the other is reported beside it (the
        # per-link exchange model cannot settle N = 2 / 4 without the links)
        todo.append((other, xp))
        if other == "users" and args.chain_beside and beside_xp is not None:
            todo.append(("users", beside_xp))
    beside_errors = []
    runs = []
    trainer = None
    for i, (part, xq) in enumerate(todo):
        if trainer is not None:
            trainer.close()
        trainer = None
        torch.cuda.empty_cache()
        if not dist_mode:   # one process: nothing to fall back to, errors are errors
            trainer = build(part, xq)
            r = measure(trainer, part, args.dense_check)
            r["xp"] = xq
            runs.append(r)
            continue
        # a run that fails on every rank alike (an RCCL communicator that will
        # not come up, memory) is reported, not fatal: the ranks agree on it and
        # the line keeps the runs that finished (the main run's failure too, as
        # long as one setting finishes)
        try:
            fail = os.environ.get("BBGR_BENCH_FAIL_BESIDE")   # the error paths' tests
            if (fail == part and i > 0) or (fail == "main" and i == 0):
                raise RuntimeError("injected failure")
            trainer = build(part, xq)
            r = measure(trainer, part, args.dense_check)
            r["xp"] = xq
            ok = 1.0
        except Exception as ex:   # noqa: BLE001
            ok, err = 0.0, f"{part} ({chain_mode(xq) if part == 'users' else 'columns'}): " \
                           f"{type(ex).__name__}: {ex}"[:400]
            log(f"[bench] rank {rank}: {'main' if i == 0 else 'beside'} run failed: {err}")
        if _allreduce(ok, dev, torch.distributed.ReduceOp.MIN) < 1.0:
            beside_errors.append(err if ok < 1.0 else f"{part}: failed on another rank")
            if trainer is not None:
                trainer.close()
            trainer = None
            continue
        runs.append(r)
    if not runs:
        raise RuntimeError("bench: every partition / chain setting failed: "
                           + " | ".join(beside_errors))
    # every rank holds the same max-over-ranks times: the same choice everywhere
    res = min(runs, key=lambda r: r["elapsed"])

    def beside(r: dict, note: str) -> dict:
        b = {k: r[k] for k in ("part", "ms_per_step", "value", "E", "final_loss")}
        if r["part"] == "users":
            b["chain_mode"] = chain_mode(r["xp"])
        b["note"] = note
        return b

    partition_beside = chain_beside = None
    others = [r for r in runs if r["part"] != res["part"]]
    if others:
        partition_beside = beside(min(others, key=lambda r: r["elapsed"]),
                                  "the other strong-scaling partition of the same graph, timed "
                                  "the same way in the same run; the faster one is the line")
    users_runs = sorted((r for r in runs if r["part"] == "users"), key=lambda r: r["elapsed"])
    if len(users_runs) == 2:
        chain_beside = beside(users_runs[1],
                              "the user-row partition's other chain setting, timed the same way "
                              "in the same run (user-row line: "
                              + chain_mode(users_runs[0]["xp"]) + ")")
        chain_beside["faster_users_ms_per_step"] = users_runs[0]["ms_per_step"]
        chain_beside["faster_chain_mode"] = chain_mode(users_runs[0]["xp"])
        if not backend_nccl:
            chain_beside["backend_note"] = ("gloo rehearsal: RCCL cannot run two ranks on one "
                                            "GPU, so the one-chain setting uses torch's "
                                            "collectives; on RCCL it runs inline through the "
                                            "C ABI's communicator")
    xsel = res.get("xp") or xp
    sel_chains = xsel.get("column_chains", 1)
    sel_parts = xsel.get("exchange_parts", args.exchange_parts)
    sel_native = {True: "stream", "stream": "stream", "inline": "inline"}.get(
        xsel.get("native_comm"), "off")
    columns = res["columns"]
    E, use_graph, timer, timer_steps = res["E"], res["use_graph"], res["timer"], res["timer_steps"]
    events_in_loop, elapsed, final_loss = res["events_in_loop"], res["elapsed"], res["final_loss"]
    counts, gathered_step, visited_step = res["counts"], res["gathered_step"], res["visited_step"]
    dense_ms, frontier_on = res["dense_ms"], res["frontier_on"]
    if dist_mode:
        del edges   # the cpu_baseline leg (rank 0, N=1 only) is the only later user
        if trainer is not None:
            trainer.close()                # the native exchange's communicator, if any
    groups = roofline_groups(timer, counts, timer_steps, count_steps, I)
    if res["dom_timer"] is not None:   # the dominant kind as timed inside the timed steps
        inloop = [g for g in roofline_groups(res["dom_timer"], counts, args.steps, count_steps, I)
                  if g["kind"] == "full" and g["side"] == "item<-user"]
        groups = [g for g in groups if not (g["kind"] == "full" and g["side"] == "item<-user")]
        groups = inloop + groups
    weak_beside = None
    if world > 1 and not weak and args.weak_beside > 0 and not sharded_gen:
        # the same machinery at fixed per-GPU work, beside the strong line:
        # every rank a full config-sized user shard over the shared items
        del trainer
        torch.cuda.empty_cache()
        try:
            weak_beside, ok = measure_weak(args, cfg, rank, world, dev, xp, frontier), 1.0
        except Exception as ex:   # noqa: BLE001
            ok, err = 0.0, f"weak: {type(ex).__name__}: {ex}"[:400]
            log(f"[bench] rank {rank}: weak beside run failed: {err}")
        if _allreduce(ok, dev, torch.distributed.ReduceOp.MIN) < 1.0:
            weak_beside = None
            beside_errors.append(err if ok < 1.0 else "weak: failed on another rank")
    # the dominant kernel: full-CSR item<-user products (spmm_kernel)
    dom = [g for g in groups if g["kind"] == "full" and g["side"] == "item<-user"]
    dom_n = sum(g["launches_per_step"] for g in dom)
    dom_ms = sum(g["avg_ms"] * g["launches_per_step"] for g in dom) / dom_n if dom_n else 0.0
    dom_bytes = (sum(g["gather_model_bytes"] * g["launches_per_step"] for g in dom) / dom_n
                 if dom_n else 0.0)
    dom_comp = (sum(g["compulsory_bytes"] * g["launches_per_step"] for g in dom) / dom_n
                if dom_n else 0.0)
    achieved = dom_bytes / (dom_ms * 1e6) if dom_ms > 0 else 0.0   # GB/s
    spmm_ms_step = sum(g["avg_ms"] * g["launches_per_step"] for g in groups)
    pmc = pmc_traffic() if (args.config == "C4" and world == 1 and not dist_mode) else None
    stp = step_traffic() if (args.config == "C4" and world == 1 and not dist_mode) else None
    # every timed launch's gather-model bytes per step (SpMMs incl. the fused
    # Adam product; the separate item Adam is not an SpMM launch and is left out)
    step_gather = sum(g["gather_model_bytes"] * g["launches_per_step"] for g in groups)
    steps_per_s = args.steps / elapsed
    if rank != 0:
        if dist_mode:
            torch.distributed.destroy_process_group()
        return
    cpu = None
    if not args.no_cpu_baseline and not dist_mode and not sharded_gen:
        log("[bench] timing the reference CPU path (bounded sample) ...")
        t_cpu = time.perf_counter()
        cpu = cpu_baseline(edges, cfg, args.config, cred, args.variant)
        cpu["affinity"] = _cpu_list_text(os.sched_getaffinity(0))
        log(f"[bench] cpu baseline took {time.perf_counter() - t_cpu:.1f}s")
    torch_ref = None
    if not args.no_torch_reference and not dist_mode and not sharded_gen and not emulate:
        # the reference's step in stock PyTorch-ROCm on this GPU (torch.sparse.mm
        # COO products, autograd, torch Adam): the like-for-like GPU baseline
        log("[bench] timing the stock-torch reference step on the GPU ...")
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from torch_sparse_step import run as torch_reference_run
        torch_ref = torch_reference_run(args.config, edges, cred, device=dev,
                                        variant=args.variant)
        torch_ref["speedup_vs_torch"] = torch_ref["step_ms"] / (1000.0 * elapsed / args.steps)
        torch_ref["note"] = ("the reference's V2 step written with its own torch calls "
                             "(sparse_coo_tensor.coalesce, torch.sparse.mm, stack.mean, "
                             "autograd, torch.optim.Adam) on this GPU, uniform batches "
                             "(tools/torch_sparse_step.py); not the oracle, not the product")
    dropin = dropin_fused = dropin_bwd = None
    if (not args.no_torch_reference and not dist_mode and not sharded_gen and not emulate
            and args.variant == "v2_pop"):
        # the same step through the drop-in module API (lightgcn_cu_pop.LightGCN on
        # the registered bbgr ops, autograd, the reference's default torch Adam)
        log("[bench] timing the drop-in module step ...")
        if os.path.join(ROOT, "tools") not in sys.path:
            sys.path.insert(0, os.path.join(ROOT, "tools"))
        from dropin_probe import run_many as dropin_run_many
        runs = dropin_run_many(args.config, edges, cred, device=dev,
                               adams=("foreach", "bbgr", "bbgr_bwd"))
        dropin, dropin_fused, dropin_bwd = runs["foreach"], runs["bbgr"], runs["bbgr_bwd"]
        common = ("Version-2 LightGCN drop-in (bbgr ops: propagate, bpr_loss and their "
                  "registered backward; get_user_item_emb() tables deferred, so bpr_loss "
                  "computes the batch rows only, bbgr::propagate_rows), input vertex order, "
                  "the reference loop's batches (epoch shuffle of the train users, "
                  "bbgr.host_sampler's positive / pop-mix negative draws; tools/dropin_probe.py)")
        dropin["note"] = common + " + torch.optim.Adam(foreach), the reference's optimizer"
        dropin_fused["note"] = (common + " + bbgr.optim.FusedAdam (same state keys), on the "
                                "same model right after the foreach timing")
        dropin_bwd["note"] = (common + " + bbgr.optim.FusedAdam(fuse_backward=True): the "
                              "optimizer step inside loss.backward(), in the last backward "
                              "products' epilogues (bbgr::bpr_adam_backward); the loop body "
                              "unchanged")
        if torch_ref is not None:
            dropin["speedup_vs_torch"] = torch_ref["step_ms"] / dropin["step_ms"]
            dropin_fused["speedup_vs_torch"] = torch_ref["step_ms"] / dropin_fused["step_ms"]
            dropin_bwd["speedup_vs_torch"] = torch_ref["step_ms"] / dropin_bwd["step_ms"]
    dense_equiv = 4 * K * E
    out = {
        "metric": "SpMM edges/sec + BPR steps/sec, |E|=50M d=64, 1/2/4/8 MI355X; %HBM roofline",
        "value": gathered_step * steps_per_s,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1000.0 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (Zipf-0.8 items, geometric user degrees; xavier init; Beta cred)",
        "config": {"workload": f"{args.config} BPR training step ({args.variant})"
                               + (f", {world} x {args.config} user shards" if weak else ""),
                   "num_users": U_job, "num_items": I, "num_edges": E,
                   "vertex_order": args.vertex_order,
                   "emb_dim": d, "num_layers": K,
                   "global_batch": B * (world if weak else 1),
                   "parallelism": (f"embedding-columns x{world} ({d // world} columns per "
                                   "rank, whole graph on every rank)" if columns else
                                   f"one column shard of {emulate} ({d // emulate} columns): "
                                   "single-GPU stand-in for one rank" if emulate else
                                   "single GPU (fused trainer)" if not dist_mode else
                                   f"user-rows x{world}"
                                   + (" (sharded trainer)" if dist_mode and world == 1 else "")
                                   + (f", {sel_chains} column chains"
                                      if dist_mode and not columns and sel_chains > 1
                                      else "")
                                   + (f", {sel_parts} item-row ranges per exchange"
                                      if dist_mode and not columns else "")
                                   + (f", collectives via the C ABI's communicator "
                                      f"({sel_native})"
                                      if dist_mode and not columns and sel_native != "off"
                                      else ""))},
        "bpr_steps_per_s": steps_per_s,
        "roofline_per_kernel": groups,
        "torch_gpu_reference": torch_ref,
        "dropin_module_step": dropin,
        "dropin_fused_adam_step": dropin_fused,
        "dropin_backward_adam_step": dropin_bwd,
        "weak_beside": weak_beside,
        "partition_beside": partition_beside,
        "beside_errors": beside_errors or None,
        "chain_beside": chain_beside,
        "allreduce_probe": ar_probe,
        "chain_rule": None if rule is None else dict(
            rule, measured=None if chain_beside is None else
            ("inline" if chain_beside["faster_chain_mode"].startswith("1 chain")
             else "two_chains")),
        "partition": ("columns" if columns else "users") if dist_mode else
                     (f"one column shard of {emulate}" if emulate else "single GPU"),
        "graph_replay": use_graph,
        "hw_queues": {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"),
                      "given": HW_QUEUES_GIVEN,
                      "note": "bench.py raises HIP's hardware queues per process to 8 (from "
                              "the given value, default 4) before the runtime starts, so the "
                              "compute, RCCL and side streams do not share one queue"},
        "value_note": "value = SpMM edges actually gathered (source row read and "
                      "multiply-added) per second, whole job: every launch's edges counted "
                      f"on the device over {count_steps} steps after the timed region "
                      "(full-CSR launches all E; frontier-masked launches only their rows' "
                      "edges with a live source)",
        "edges_gathered_per_step": gathered_step,
        "edges_visited_per_step": visited_step,
        "reference_equivalent_edges_per_s": dense_equiv * steps_per_s,
        "reference_equivalent_note": "4*K*E per step (the reference's dense step: 2K "
                                     "products forward, 2K backward) / this step time: NOT "
                                     "edges traversed here",
        "dense_ms_per_step": dense_ms,
        "dense_edges_per_s": (dense_equiv / (dense_ms / 1e3)) if dense_ms else None,
        "dense_note": "same trainer, frontier sparsity off (every SpMM over the full CSR; "
                      "loss, gradients and updates equal): timed after the main loop; "
                      "dense_edges_per_s = 4*K*E traversed per dense step",
        "frontier": {"enabled": frontier_on,
                     "full_sequence_ms": [
                         {"rows": r, "nnz": z, "avg_ms": ms}
                         for r, z, ms in timer.sequence("full", timer_steps)],
                     "adam_sequence_ms": [
                         {"rows": r, "nnz": z, "avg_ms": ms}
                         for r, z, ms in timer.sequence("adam", timer_steps)
                         + timer.sequence("adam_side", timer_steps)],
                     "masked_sequence_ms": [
                         {"rows": r, "nnz": z, "avg_ms": ms}
                         for r, z, ms in timer.sequence("masked", timer_steps)]},
        "spmm_ms_per_step": spmm_ms_step,
        "final_loss": final_loss,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": None if pmc is None else pmc.get("hbm_bytes_per_launch_corrected"),
                     "kernel": "bbgr::spmm_kernel (split rows finished in-launch): full-CSR item<-user "
                               "product, the largest share of step time",
                     "algorithmic_bytes_per_launch": dom_bytes,
                     "algorithmic_model": "gather model E*(4+4+4d) + R*(4+4d) (SURVEY §8(d))",
                     "compulsory_bytes_per_launch": dom_comp,
                     "compulsory_frac": (dom_comp / (dom_ms * 1e6) / HBM_PEAK_GBS) if dom_ms else None,
                     "compulsory_model": "E*8 + C*4d + R*(4+4d), C = source rows (SURVEY §8(d)(ii))",
                     "avg_launch_ms": dom_ms, "launches_per_step": dom_n,
                     "events": ("HIP events on the launching stream, inside the timed steps "
                                "(this kernel's launches only; the other kinds over "
                                f"{timer_steps} eager steps after the timed region)"
                                if events_in_loop else
                                f"HIP events over {timer_steps} eager steps after the timed "
                                "region" + (" (timed steps are graph replays)" if use_graph
                                            else "")),
                     "traffic_unit": "HBM bytes per launch, 2*FETCH_SIZE+WRITE_SIZE (rocprofv3 "
                                     "PMC, gfx950 correction); counts Infinity-Cache hits",
                     "traffic_source": None if pmc is None else
                     {k: pmc.get(k) for k in ("tag", "commit", "kernel", "avg_us", "dispatches")},
                     "cache_assisted": achieved > HBM_GATHER_CEILING_GBS,
                     "cache_assisted_rule": "gather-model GB/s above 5800, the guide's "
                                            "measured rate for random whole-row gathers "
                                            "from HBM (MI355X_MICROARCH.md)",
                     "step_gather_model_GBps": step_gather / (1e6 * 1000.0 * elapsed
                                                              / args.steps),
                     "step_gather_model_note": "the SpMM launches' gather-model bytes per "
                                               "step / ms_per_step (zero-reuse model: can "
                                               "exceed the HBM peak where rows are re-read "
                                               "from caches)",
                     "step_traffic_bytes": None if stp is None else
                     stp["hbm_bytes_per_step_corrected"],
                     "step_traffic_GBps": None if stp is None else
                     stp["hbm_bytes_per_step_corrected"] / (1e6 * 1000.0 * elapsed / args.steps),
                     "step_traffic_frac": None if stp is None else
                     stp["hbm_bytes_per_step_corrected"] / (1e6 * 1000.0 * elapsed / args.steps)
                     / HBM_PEAK_GBS,
                     "step_traffic_source": None if stp is None else
                     {k: stp.get(k) for k in ("tag", "commit", "steps", "kernel_us_per_step_pmc",
                                              "source")}},
        "cpu_baseline": None if cpu is None else {k: v for k, v in cpu.items() if k != "step_s"},
        # last: the compact figures, where the driver's stdout tail keeps them
        "step_summary": step_summary(1000.0 * elapsed / args.steps, dense_ms, torch_ref, dropin,
                                     dropin_fused, dropin_bwd),
    }
    print(json.dumps(out), file=out_stream, flush=True)
    if dist_mode:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
