"""Full-size parity at the BASELINE workloads (north_star:
"layer-K embeddings match the reference forward to 1e-5 rel").

The float64 oracle cannot hold a 50M/500M-edge propagation in host memory,
so each product is checked on sampled output rows instead: the GPU computes
layer k from its own layer k-1 (the drop-in operators' products, the
torch.sparse.mm calls of the reference's propagate loop), and the oracle
recomputes ~10k of layer k's rows in float64 from their CSR neighbourhoods
in the host edge list, with the reference's fp32 operator values
(oracle/ref_numpy.edge_weights, from host-side degrees). Every layer and
side is checked; then the fused training-path forward (degree-ordered graph,
the bench's layout) is checked against the float64 layer mean of the same
rows; at C4 the first training step's weight gradients are checked the same
way through every backward product.

Sampled rows: random rows of each side, plus high-degree rows (the chunked,
fixed-order long-row path) up to an edge budget, plus (gradient test) the
batch rows. Tolerance: normwise relative <= 1e-5 and max-abs <= 1e-5*max|ref|
over the sampled rows.

  C1  lightgcn.py symmetric path, 943 x 1682, 100K edges, d=64, K=3:
      whole tables against tests/golden/golden_c1.npz (every layer, final,
      BPR loss, gradient of emb.weight)
  C3  lightgcn_cu.py Jacobi path, Beta credibility, 5M x 1M, 50M edges, d=128, K=3
  C4  Version-2 GS path, Beta credibility, 5M x 1M, 50M edges, d=64, K=3
      (+ the first training step's gradients, B=8192)
  C5  GS path, 10M x 2M, 500M edges, d=256, K=4 (the 8-GPU config, on one GPU)
"""
import multiprocessing as mp
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from bbgr.synthetic import (CONFIGS, CONFIG_SEED, config_edges,  # noqa: E402
                            shard_edges_strong, synthetic_credibility)
from oracle import ref_numpy as R  # noqa: E402

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


_EDGES = {}


def workload_edges(name: str) -> np.ndarray:
    """The config's synthetic graph. C5 (500M edges) is drawn as the union of
    its 8 user shards (the graph the 8-GPU run trains on), in parallel. C4's
    graph is kept for the gradient test."""
    if name in _EDGES:
        return _EDGES[name]
    if name != "C5":
        e = config_edges(name)
    else:
        with mp.get_context("spawn").Pool(8) as pool:
            parts = pool.map(_c5_shard, [(r, 8) for r in range(8)])
        e = np.concatenate(parts, axis=1)
    if name == "C4":
        _EDGES[name] = e
    return e


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


class SideEdges:
    """The host edges whose OUTPUT row (on one side) is in a sampled set."""

    def __init__(self, out_ids: np.ndarray, src_ids: np.ndarray, n_out: int, sel: np.ndarray,
                 w_all_fn):
        m = np.zeros(n_out, bool)
        m[sel] = True
        k = np.flatnonzero(m[out_ids])
        self.sel = sel
        self.rows = out_ids[k].astype(np.int64)
        self.cols = src_ids[k].astype(np.int64)
        self.k = k
        self.w = w_all_fn(k)     # fp32 values of these edges (oracle expressions)


def oracle_rows(side: SideEdges, x_gpu: torch.Tensor, chunk: int = 1 << 20) -> np.ndarray:
    """float64 rows side.sel of (M x) from the GPU's x (its fp32 values)."""
    out = np.zeros((side.sel.size, x_gpu.shape[1]), np.float64)
    for a in range(0, side.rows.size, chunk):
        cols = side.cols[a:a + chunk]
        uniq, inv = np.unique(cols, return_inverse=True)
        xs = x_gpu[torch.from_numpy(uniq).to(x_gpu.device)].cpu().numpy()
        out += R.rows_product(side.sel, side.rows[a:a + chunk], cols,
                              side.w[a:a + chunk], xs[inv])
    return out


def gpu_rows(t: torch.Tensor, sel: np.ndarray) -> np.ndarray:
    return t[torch.from_numpy(sel).to(t.device)].double().cpu().numpy()


KINDS = {   # config -> operator family, drop-in builder, fused-trainer variant
    "C3": ("j", "cu_fair"),
    "C4": ("gs", "v2_pop"),
    "C5": ("gs", "v2_pop"),
}


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


def run_layers(name, check_grads=False):
    c = CONFIGS[name]
    U, I, d, K = c["num_users"], c["num_items"], c["emb_dim"], c["num_layers"]
    kind, variant = KINDS[name]
    e = workload_edges(name)
    assert e.shape[1] == c["num_edges"]
    cred = synthetic_credibility(U, CONFIG_SEED[name], "beta")
    deg_u, deg_i = R.degrees(e, U, I)
    rng = np.random.default_rng(CONFIG_SEED[name])
    budget = 2_000_000 if d <= 128 else 1_000_000
    sel_u = sample_rows(deg_u.astype(np.int64), rng, N_SAMPLE, budget)
    sel_i = sample_rows(deg_i.astype(np.int64), rng, N_SAMPLE, budget)

    def w_fn(k):
        return R.edge_weights(kind, e[0, k], e[1, k], deg_u, deg_i, cred)

    ue = SideEdges(e[0], e[1], U, sel_u, lambda k: w_fn(k)[0])   # user rows <- items
    ie = SideEdges(e[1], e[0], I, sel_i, lambda k: w_fn(k)[1])   # item rows <- users
    item_op, user_op = drop_in_operators(kind, e, U, I, cred)
    u0, i0 = device_tables(U, I, d)
    us, is_ = [gpu_rows(u0, sel_u)], [gpu_rows(i0, sel_i)]
    u, i = u0, i0
    for k in range(1, K + 1):
        if kind == "gs":     # Version-2:482-487: items first, users from the NEW items
            i_new = item_op.mm(u)
            u_new = user_op.mm(i_new)
            want_i, want_u = oracle_rows(ie, u), oracle_rows(ue, i_new)
        else:                # lightgcn_cu.py:429-447: both sides from layer k-1
            i_new, u_new = item_op.mm(u), user_op.mm(i)
            want_i, want_u = oracle_rows(ie, u), oracle_rows(ue, i)
        got_i, got_u = gpu_rows(i_new, sel_i), gpu_rows(u_new, sel_u)
        assert_parity(got_i, want_i, f"{name} {kind} item layer {k}")
        assert_parity(got_u, want_u, f"{name} {kind} user layer {k}")
        us.append(got_u)
        is_.append(got_i)
        if k > 1:
            del u, i
        u, i = u_new, i_new
    del u, i, item_op, user_op
    torch.cuda.empty_cache()
    # the fused training-path forward on the degree-ordered graph (bench layout)
    from bbgr.graph import BipartiteGraph
    from bbgr.trainer import FusedTrainer
    graph = BipartiteGraph(e, U, I, DEV, vertex_order="degree")
    tr = FusedTrainer(graph, variant, cred=cred, emb_dim=d, num_layers=K,
                      batch_size=c["batch"], u0=u0, i0=i0, fuse_adam=not check_grads)
    del u0, i0
    uf, itf = tr.forward()
    assert_parity(gpu_rows(uf, sel_u), np.mean(us, 0), f"{name} fused forward u_final")
    assert_parity(gpu_rows(itf, sel_i), np.mean(is_, 0), f"{name} fused forward i_final")
    out = dict(e=e, cred=cred, U=U, I=I, d=d, K=K, kind=kind, tr=tr, uf=uf, itf=itf,
               deg_u=deg_u, deg_i=deg_i, rng=rng, budget=budget)
    return out


@pytest.mark.parametrize("name", ["C3", "C4", "C5"])
def test_every_layer_and_fused_forward_full_size(name):
    run_layers(name)
    torch.cuda.empty_cache()


def test_c4_first_training_step_gradients_full_size():
    """The first fused training step at C4 (frontier masks, degree order,
    B=8192 pop-mix batch): loss vs the float64 BPR of the step's batch on the
    GPU final tables, and grad(u0) / grad(i0) on sampled + batch rows vs the
    backward chain evaluated product by product (each product checked against
    the float64 oracle from its GPU input)."""
    from bbgr.lightgcn_cu_pop import build_message_passing_mats
    from bbgr.propagate import spmm
    from bbgr.trainer import _input_rows
    w = run_layers("C4", check_grads=True)
    tr, e, cred, U, I, d, K = (w[k] for k in ("tr", "e", "cred", "U", "I", "d", "K"))
    deg_u, deg_i, rng, budget = w["deg_u"], w["deg_i"], w["rng"], w["budget"]
    uf, itf = w["uf"], w["itf"]                      # forward of the step's weights (input ids)
    u0 = _input_rows(tr.graph.user_order, tr.user_w).clone()
    i0 = _input_rows(tr.graph.item_order, tr.item_w).clone()
    loss = float(tr.step())
    users, pos, neg = (x.cpu().numpy() for x in tr.batch())
    g_u0 = _input_rows(tr.graph.user_order, tr.g_u0)
    g_i0 = _input_rows(tr.graph.item_order, tr.g_i0)
    # float64 BPR on compact tables of the batch rows (Version-2:495-508)
    bu, inv_u = np.unique(users, return_inverse=True)
    bi, inv_i = np.unique(np.concatenate([pos, neg]), return_inverse=True)
    B = users.size
    want_loss, g = R.bpr_loss(gpu_rows(uf, bu), gpu_rows(itf, bi), gpu_rows(u0, bu),
                              gpu_rows(i0, bi), inv_u, inv_i[:B], inv_i[B:], tr.reg)
    assert abs(loss - want_loss) <= TOL * abs(want_loss), (loss, want_loss)
    gU = torch.zeros(U, d, device=DEV)
    gI = torch.zeros(I, d, device=DEV)
    gU[torch.from_numpy(bu).to(DEV)] = torch.from_numpy(g["g_uf"]).float().to(DEV)
    gI[torch.from_numpy(bi).to(DEV)] = torch.from_numpy(g["g_if"]).float().to(DEV)
    # sampled rows now include the batch rows (the BPR terms land there)
    sel_u = sample_rows(deg_u.astype(np.int64), rng, N_SAMPLE, budget, extra=bu[:2000])
    sel_i = sample_rows(deg_i.astype(np.int64), rng, N_SAMPLE, budget, extra=bi[:2000])

    def w_fn(k):
        return R.edge_weights("gs", e[0, k], e[1, k], deg_u, deg_i, cred)

    # transposed products: M_ui^T (item rows <- users, values of M_ui) and
    # M_iu^T (user rows <- items, values of M_iu)
    it_side = SideEdges(e[1], e[0], I, sel_i, lambda k: w_fn(k)[0])
    us_side = SideEdges(e[0], e[1], U, sel_u, lambda k: w_fn(k)[1])
    M_ui, M_iu = build_message_passing_mats(e, U, I, torch.from_numpy(cred).to(DEV), DEV)
    pair = M_iu.pair

    def T(prod, x):
        y = torch.empty(prod.csr.n_rows, d, device=DEV)
        spmm(prod, x, True, y=y, y_scale=prod.out_scale)
        return y

    gl = 1.0 / (K + 1)
    gUs, gIs = gU * gl, gI * gl
    Gu = gUs
    for k in range(K, 0, -1):      # autograd of Version-2:482-489
        t_i = T(pair.bwd_item, Gu)
        assert_parity(gpu_rows(t_i, sel_i), oracle_rows(it_side, Gu), f"C4 M_ui^T product {k}")
        Gi = gIs + t_i
        t_u = T(pair.bwd_user, Gi)
        assert_parity(gpu_rows(t_u, sel_u), oracle_rows(us_side, Gi), f"C4 M_iu^T product {k}")
        Gu = gUs + t_u
    ego_u = np.zeros((sel_u.size, d))
    ego_i = np.zeros((sel_i.size, d))
    pu = {int(r): j for j, r in enumerate(bu)}
    pi = {int(r): j for j, r in enumerate(bi)}
    for j, r in enumerate(sel_u):
        if int(r) in pu:
            ego_u[j] = g["g_ue"][pu[int(r)]]
    for j, r in enumerate(sel_i):
        if int(r) in pi:
            ego_i[j] = g["g_ie"][pi[int(r)]]
    assert_parity(gpu_rows(g_u0, sel_u), gpu_rows(Gu, sel_u) + ego_u, "C4 grad u0")
    assert_parity(gpu_rows(g_i0, sel_i), gpu_rows(gIs, sel_i) + ego_i, "C4 grad i0")


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
