"""Full-size parity at the BASELINE workloads (north_star:
"layer-K embeddings match the reference CPU/PyTorch forward to 1e-5 rel on
identical inputs").

Every GPU result here is compared with a float64 chain computed on the host
from the SAME u0 / i0 (oracle/chain64.py over oracle/csrc/chain64.c): the
reference's K-layer propagation (Version-2/lighgcn_cu_pop.py:472-490,
lightgcn_cu.py:420-448) with the reference's fp32 operator values
(oracle/ref_numpy.edge_weights, host-side degrees), in float64, every layer.
No assertion compares the GPU with its own intermediates. Checked per config:

  * every layer k and side of the drop-in operators' chain (the
    torch.sparse.mm calls of the reference's propagate loop, BipartiteOperator.mm);
  * the drop-in module's final tables (LightGCN.propagate() /
    CredLightGCN.final_embeddings(), i.e. the bbgr::propagate op);
  * the fused training path's forward (degree-ordered graph, the bench layout);
  * C3 / C4 / C5: the first fused training step's loss (float64 BPR of the
    step's batch on the float64 final tables; C3 with the lambda_fair term of
    lightgcn_cu.py:637-648) and grad(u0) / grad(i0) (float64 adjoint chain of
    that BPR gradient plus the ego-L2 rows: Version-2:862 / lightgcn_cu.py:650
    autograd), Jacobi order for C3, Gauss-Seidel for C4 / C5.

Compared rows: random rows of each side, the heaviest rows up to an edge
budget (the chunked, fixed-order long-row path) and (gradients) the batch
rows. Tolerance: normwise relative <= 1e-5 and max-abs <= 1e-5*max|ref| over
the compared rows. C5 (500M edges, d=256) runs its float64 chain on 16 of the
256 columns (all 256 columns at 500M edges would take ~10 min of host time):
its u0 / i0 are drawn at full width and then zeroed outside those 16 random
columns. Propagation acts on each column alone, so the checked columns are
exactly the full-width chain's; and the BPR dot products then involve only
those columns, so the float64 loss and gradient of the 16-column chain ARE
the full-width step's (the other 240 columns of every gradient are 0, also
checked). The d=256 kernels run unchanged over all 256 columns.

  C1  lightgcn.py symmetric path, 943 x 1682, 100K edges, d=64, K=3:
      whole tables against tests/golden/golden_c1.npz (every layer, final,
      BPR loss, gradient of emb.weight)
  C3  lightgcn_cu.py Jacobi path, Beta credibility, 5M x 1M, 50M edges, d=128, K=3
  C4  Version-2 GS path, Beta credibility, 5M x 1M, 50M edges, d=64, K=3
      (+ the first training step's loss and gradients, B=8192)
  C5  GS path, 10M x 2M, 500M edges, d=256, K=4 (the 8-GPU config, on one GPU)
"""
import multiprocessing as mp
import os
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from bbgr.synthetic import (CONFIGS, CONFIG_SEED, config_edges,  # noqa: E402
                            shard_edges_strong, synthetic_credibility)
from oracle import ref_numpy as R  # noqa: E402
from oracle.chain64 import Chain64  # noqa: E402

DEV = "cuda"
TOL = 1e-5
HERE = os.path.dirname(os.path.abspath(__file__))
N_SAMPLE = 10_000


def assert_parity(got, ref, what, tol=TOL):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    nrm = np.linalg.norm(ref)
    err = np.linalg.norm(got - ref)
    assert err <= tol * max(nrm, 1e-30), f"{what}: normwise rel err {err / max(nrm, 1e-30):.3e}"
    mx = np.abs(ref).max() if ref.size else 0.0
    assert np.abs(got - ref).max() <= tol * max(mx, 1e-30), \
        f"{what}: max-abs err {np.abs(got - ref).max():.3e} vs {tol * mx:.3e}"


# ---------------------------------------------------------------------------
# workloads
# ---------------------------------------------------------------------------
def _c5_shard(rank_world):
    rank, world = rank_world
    e, lo, hi = shard_edges_strong("C5", rank, world)
    e[0] += lo
    return e


def workload_edges(name: str) -> np.ndarray:
    """The config's synthetic graph. C5 (500M edges) is drawn as the union of
    its 8 user shards (the graph the 8-GPU run trains on), in parallel."""
    if name != "C5":
        return config_edges(name)
    with mp.get_context("spawn").Pool(8) as pool:
        parts = pool.map(_c5_shard, [(r, 8) for r in range(8)])
    return np.concatenate(parts, axis=1)


def device_tables(U, I, d, seed=42):
    """xavier_uniform_ tables drawn on the device (a 10M x 256 table is 10 GB)."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    au, ai = (6.0 / (U + d)) ** 0.5, (6.0 / (I + d)) ** 0.5
    u0 = (torch.rand(U, d, generator=g, device=DEV) * 2 - 1) * au
    i0 = (torch.rand(I, d, generator=g, device=DEV) * 2 - 1) * ai
    return u0, i0


def sample_rows(deg: np.ndarray, rng, n: int, budget: int, extra=None) -> np.ndarray:
    """n random rows + the heaviest rows whose degrees fit `budget` edges
    together (they run the chunked long-row path) + `extra` rows."""
    rows = rng.choice(deg.size, size=min(n, deg.size), replace=False)
    order = np.argsort(-deg, kind="stable")
    heavy, used = [], 0
    for r in order[: 4096]:
        if used + deg[r] <= budget:
            heavy.append(r)
            used += int(deg[r])
    parts = [rows, np.asarray(heavy, np.int64)]
    if extra is not None:
        parts.append(np.asarray(extra, np.int64))
    return np.unique(np.concatenate(parts))


def gpu_rows(t: torch.Tensor, sel: np.ndarray, cols=None) -> np.ndarray:
    r = t[torch.from_numpy(np.asarray(sel, np.int64)).to(t.device)]
    if cols is not None:
        r = r[:, torch.from_numpy(cols).to(t.device)]
    return r.double().cpu().numpy()


def host_cols(t: torch.Tensor, cols=None) -> np.ndarray:
    """The fp32 device table (or its `cols` columns) as a float64 host array."""
    if cols is not None:
        t = t[:, torch.from_numpy(cols).to(t.device)]
    return t.double().cpu().numpy()


KINDS = {   # config -> operator family, propagation order, fused-trainer variant
    "C3": ("j", "jacobi", "cu_fair"),
    "C4": ("gs", "gs", "v2_pop"),
    "C5": ("gs", "gs", "v2_pop"),
}
CHAIN_COLS = {"C5": 16}   # float64 chain on a column subset (see the docstring)


def drop_in_operators(kind, e, U, I, cred):
    """(item<-user, user<-item) operators from the reference-named builders."""
    if kind == "gs":
        from bbgr.lightgcn_cu_pop import build_message_passing_mats
        M_ui, M_iu = build_message_passing_mats(e, U, I, torch.from_numpy(cred).to(DEV), DEV)
        return M_iu, M_ui
    if kind == "j":
        from bbgr.lightgcn_cu import build_cred_weighted_mats
        item_from_user, user_from_item, _ = build_cred_weighted_mats(e, U, I, cred, DEV)
        return item_from_user, user_from_item
    raise ValueError(kind)


def drop_in_model(kind, e, U, I, d, K, cred, u0, i0):
    """The reference-named module (Version-2 LightGCN / lightgcn_cu
    CredLightGCN) on its own builders, weights set to u0 / i0; returns its
    final tables (the caller's propagate() / final_embeddings())."""
    if kind == "gs":
        from bbgr.lightgcn_cu_pop import LightGCN as Model, build_message_passing_mats
        ops = build_message_passing_mats(e, U, I, torch.from_numpy(cred).to(DEV), DEV)
    else:
        from bbgr.lightgcn_cu import CredLightGCN as Model, build_cred_weighted_mats
        ops = build_cred_weighted_mats(e, U, I, cred, DEV)[:2]
    with torch.device(DEV):   # (the module's own xavier init on the device: C5 is 12 GB)
        m = Model(U, I, d, K, *ops)
    with torch.no_grad():
        m.user_emb.weight.copy_(u0)
        m.item_emb.weight.copy_(i0)
        uf, itf = m.propagate() if kind == "gs" else m.final_embeddings()
    return m, uf, itf


def _progress(t0, what):
    """A line per stage (a C5 run takes minutes; run with -s to see them)."""
    print(f"[fullsize {time.perf_counter() - t0:7.1f} s] {what}", flush=True)


def run_full(name, check_grads=False):
    """Every GPU form of the config's forward against the float64 chain from
    the same u0 / i0; returns the state the gradient check continues from."""
    t0 = time.perf_counter()
    c = CONFIGS[name]
    U, I, d, K = c["num_users"], c["num_items"], c["emb_dim"], c["num_layers"]
    kind, order, variant = KINDS[name]
    e = workload_edges(name)
    assert e.shape[1] == c["num_edges"]
    cred = synthetic_credibility(U, CONFIG_SEED[name], "beta")
    rng = np.random.default_rng(CONFIG_SEED[name])
    cols = None
    if name in CHAIN_COLS:
        cols = np.sort(rng.choice(d, CHAIN_COLS[name], replace=False))
    _progress(t0, f"{name}: graph drawn ({e.shape[1]} edges)")
    chain = Chain64(e, U, I, kind, cred)
    _progress(t0, f"{name}: float64 operator CSRs built")
    budget = 2_000_000 if d <= 128 else 1_000_000
    sel_u = sample_rows(chain.deg_u.astype(np.int64), rng, N_SAMPLE, budget)
    sel_i = sample_rows(chain.deg_i.astype(np.int64), rng, N_SAMPLE, budget)
    u0, i0 = device_tables(U, I, d)
    if cols is not None:   # tables supported on the chain's columns (docstring)
        off = torch.ones(d, dtype=torch.bool, device=DEV)
        off[torch.from_numpy(cols).to(DEV)] = False
        u0[:, off] = 0.0
        i0[:, off] = 0.0
    u0h, i0h = host_cols(u0, cols), host_cols(i0, cols)
    ruf, ritf, lay_u, lay_i = chain.forward(u0h, i0h, K, order, keep_u=sel_u, keep_i=sel_i)
    _progress(t0, f"{name}: float64 chain done ({'all' if cols is None else len(cols)} columns)")
    tag = f"{name} {kind}"

    # (1) the drop-in operators' layer chain (the reference's propagate loop)
    item_op, user_op = drop_in_operators(kind, e, U, I, cred)
    u, i = u0, i0
    for k in range(1, K + 1):
        if order == "gs":      # Version-2:482-487: items first, users from the NEW items
            i_new = item_op.mm(u)
            u_new = user_op.mm(i_new)
        else:                  # lightgcn_cu.py:429-447: both sides from layer k-1
            i_new, u_new = item_op.mm(u), user_op.mm(i)
        assert_parity(gpu_rows(i_new, sel_i, cols), lay_i[k], f"{tag} item layer {k}")
        assert_parity(gpu_rows(u_new, sel_u, cols), lay_u[k], f"{tag} user layer {k}")
        if k > 1:
            del u, i
        u, i = u_new, i_new
    del u, i, item_op, user_op
    torch.cuda.empty_cache()
    _progress(t0, f"{name}: drop-in operator layers checked")

    # (2) the drop-in module's final tables (bbgr::propagate)
    m, uf, itf = drop_in_model(kind, e, U, I, d, K, cred, u0, i0)
    assert_parity(gpu_rows(uf, sel_u, cols), ruf[sel_u], f"{tag} drop-in module u_final")
    assert_parity(gpu_rows(itf, sel_i, cols), ritf[sel_i], f"{tag} drop-in module i_final")
    del m, uf, itf
    torch.cuda.empty_cache()
    _progress(t0, f"{name}: drop-in module finals checked")

    # (3) the fused training path's forward (degree-ordered graph, bench layout)
    from bbgr.graph import BipartiteGraph
    from bbgr.trainer import FusedTrainer
    graph = BipartiteGraph(e, U, I, DEV, vertex_order="degree")
    tr = FusedTrainer(graph, variant, cred=cred, emb_dim=d, num_layers=K,
                      batch_size=c["batch"], u0=u0, i0=i0, fuse_adam=not check_grads,
                      lambda_fair=FAIR.get(name, 0.0))
    del u0, i0
    uf, itf = tr.forward()
    assert_parity(gpu_rows(uf, sel_u, cols), ruf[sel_u], f"{tag} fused forward u_final")
    assert_parity(gpu_rows(itf, sel_i, cols), ritf[sel_i], f"{tag} fused forward i_final")
    del uf, itf
    _progress(t0, f"{name}: fused-trainer forward checked")
    if not check_grads:
        return None
    return dict(e=e, U=U, I=I, d=d, K=K, tr=tr, chain=chain, ruf=ruf, ritf=ritf,
                u0h=u0h, i0h=i0h, rng=rng, budget=budget, cols=cols, order=order)


# lambda_fair of the first-step check: lightgcn_cu.py:61 ("set e.g. 1e-2 to
# enable Eq (3.27)"); the Jacobi family is the only one with the term
FAIR = {"C3": 1e-2}


def first_step_grads(name: str):
    """The config's forward as in run_full, then the first fused training step
    (frontier masks, degree order, B=8192 batch of the variant's sampler,
    separate Adam so the weight gradients are kept): its loss against the
    float64 BPR (Version-2:495-508; + lambda_fair * mean(pop[pos] * s+) with
    pop = deg_i / max deg_i, lightgcn_cu.py:583-584, 637-648) of the step's
    batch on the float64 final tables, and grad(u0) / grad(i0) on sampled +
    batch rows against the float64 adjoint chain of that BPR gradient (the
    family's own order) plus the ego-L2 rows."""
    from bbgr.trainer import _input_rows
    t0 = time.perf_counter()
    w = run_full(name, check_grads=True)
    tr, chain, U, I, d, K = (w[k] for k in ("tr", "chain", "U", "I", "d", "K"))
    ruf, ritf, u0h, i0h, cols = w["ruf"], w["ritf"], w["u0h"], w["i0h"], w["cols"]
    lam = FAIR.get(name, 0.0)
    pop = None
    if lam:
        assert tr.pop is not None and tr.lambda_fair == lam
        pop = chain.deg_i / max(float(chain.deg_i.max()), 1.0)
    loss = float(tr.step())
    _progress(t0, f"{name}: first fused step done")
    users, pos, neg = (x.cpu().numpy() for x in tr.batch())
    g_u0 = _input_rows(tr.graph.user_order, tr.g_u0)
    g_i0 = _input_rows(tr.graph.item_order, tr.g_i0)
    bu, inv_u = np.unique(users, return_inverse=True)
    bi, inv_i = np.unique(np.concatenate([pos, neg]), return_inverse=True)
    B = users.size
    want_loss, g = R.bpr_loss(ruf[bu], ritf[bi], u0h[bu], i0h[bi], inv_u, inv_i[:B],
                              inv_i[B:], tr.reg, None if pop is None else pop[bi], lam)
    assert abs(loss - want_loss) <= TOL * abs(want_loss), (loss, want_loss)
    dc = u0h.shape[1]
    gU = np.zeros((U, dc))
    gI = np.zeros((I, dc))
    gU[bu] = g["g_uf"]
    gI[bi] = g["g_if"]
    Gu, Gi = chain.backward(gU, gI, K, w["order"])
    del gU, gI
    Gu[bu] += g["g_ue"]
    Gi[bi] += g["g_ie"]
    _progress(t0, f"{name}: float64 adjoint chain done")
    sel_u = sample_rows(chain.deg_u.astype(np.int64), w["rng"], N_SAMPLE, w["budget"],
                        extra=bu[:2000])
    sel_i = sample_rows(chain.deg_i.astype(np.int64), w["rng"], N_SAMPLE, w["budget"],
                        extra=bi[:2000])
    assert_parity(gpu_rows(g_u0, sel_u, cols), Gu[sel_u], f"{name} grad u0")
    assert_parity(gpu_rows(g_i0, sel_i, cols), Gi[sel_i], f"{name} grad i0")
    if cols is not None:   # the columns off the tables' support carry no gradient
        off = np.setdiff1d(np.arange(d), cols)
        for t_, sel, what in ((g_u0, sel_u, "u0"), (g_i0, sel_i, "i0")):
            assert not np.any(gpu_rows(t_, sel, off)), f"{name} grad {what} off-support columns"


@pytest.mark.parametrize("name", ["C3", "C5"])
def test_full_chain_every_layer_finals_and_first_step_grads(name):
    first_step_grads(name)
    torch.cuda.empty_cache()


def test_c4_full_chain_and_first_training_step():
    """C4 forward as in run_full, then the first fused training step (B=8192
    pop-mix batch): loss and grad(u0) / grad(i0) against the float64 chain."""
    first_step_grads("C4")
    torch.cuda.empty_cache()


# ---------------------------------------------------------------------------
# C1: whole tables against the committed golden (lightgcn.py path)
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def c1():
    return dict(np.load(os.path.join(HERE, "golden", "golden_c1.npz")))


def t(a, dtype=torch.float32):
    return torch.as_tensor(np.asarray(a)).to(DEV, dtype)


def test_c1_symmetric_path_every_layer_loss_and_grad_vs_golden(c1):
    from bbgr.lightgcn import LightGCN, build_norm_adj
    from bbgr.operators import ITEM_FROM_USER, USER_FROM_ITEM, BipartiteOperator
    U, I, E, d, K = (int(x) for x in c1["meta"])
    e = c1["edges"]
    A = build_norm_adj(e, U, I, DEV)
    item_op = BipartiteOperator(A.pair, ITEM_FROM_USER)
    user_op = BipartiteOperator(A.pair, USER_FROM_ITEM)
    u, i = t(c1["u0"]), t(c1["i0"])
    for k in range(1, K + 1):      # lightgcn.py:320-325 on the two blocks
        u, i = user_op.mm(i), item_op.mm(u)
        assert_parity(torch.cat([u, i]).double().cpu().numpy(), c1[f"sym_x{k}"],
                      f"C1 sym layer {k}")
    model = LightGCN(U, I, d, K, A).to(DEV)
    with torch.no_grad():
        model.emb.weight.copy_(t(np.concatenate([c1["u0"], c1["i0"]])))
    uf, itf = model.get_user_item_emb()
    assert_parity(torch.cat([uf, itf]).detach().double().cpu().numpy(), c1["sym_xf"],
                  "C1 sym final")
    users, pos, neg = (t(c1[k], torch.int64) for k in ("users", "pos", "neg"))
    loss = model.bpr_loss(users, pos, neg, uf, itf, 1e-4)
    assert abs(float(loss.detach()) - float(c1["sym_loss"])) <= TOL * float(c1["sym_loss"])
    loss.backward()
    assert_parity(model.emb.weight.grad.double().cpu().numpy(), c1["sym_grad_emb"],
                  "C1 grad emb.weight")


@pytest.mark.parametrize("variant", ["gs", "method_a", "j"])
def test_c1_other_families_final_tables_vs_golden(c1, variant):
    U, I, E, d, K = (int(x) for x in c1["meta"])
    e, cred = c1["edges"], c1["cred"]
    if variant == "j":
        from bbgr.lightgcn_cu import CredLightGCN, build_cred_weighted_mats
        a, b, _ = build_cred_weighted_mats(e, U, I, cred, DEV)
        model = CredLightGCN(U, I, d, K, a, b).to(DEV)
    else:
        if variant == "gs":
            from bbgr.lightgcn_cu_pop import LightGCN, build_message_passing_mats
        else:
            from bbgr.lightgcn_cu_pop_long_tail_exposure import (LightGCN,
                                                                  build_message_passing_mats)
        M_ui, M_iu = build_message_passing_mats(e, U, I, t(cred), DEV)
        model = LightGCN(U, I, d, K, M_ui, M_iu).to(DEV)
    with torch.no_grad():
        model.user_emb.weight.copy_(t(c1["u0"]))
        model.item_emb.weight.copy_(t(c1["i0"]))
    if variant == "j":
        uf, itf = model.final_embeddings()
    else:
        uf, itf = model.propagate()
    key = {"gs": "gs", "method_a": "ma", "j": "j"}[variant]
    assert_parity(uf.detach().double().cpu().numpy(), c1[f"{key}_uf"], f"C1 {variant} u_final")
    assert_parity(itf.detach().double().cpu().numpy(), c1[f"{key}_if"], f"C1 {variant} i_final")


def test_c1_sharded_batch_capped_at_train_users():
    """A shard with fewer train users than the requested batch (C1's 943 users,
    B=4096) takes every train user once per step: no repeated rows, full
    shapes for the all-gathers (the batch used to be padded with
    repeats and an uninitialised tail)."""
    import torch.distributed as dist
    from bbgr.distributed import ShardedTrainer
    c = CONFIGS["C1"]
    U, I = c["num_users"], c["num_items"]
    e = config_edges("C1")
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29571")
        dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        tr = ShardedTrainer.from_global_edges(e, U, I, "v2_pop", cred=None, batch_size=4096,
                                              device=DEV)
        n = int(np.unique(e[0]).size)
        assert tr.B_local == n
        for _ in range(3):
            loss = float(tr.step())
            users = tr._last_users.cpu().numpy()
            assert users.size == n and np.unique(users).size == n
            assert np.isfinite(loss)
    finally:
        dist.destroy_process_group()
