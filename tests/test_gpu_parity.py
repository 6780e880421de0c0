"""GPU parity tests: the HIP path (libbbgr.so through the C ABI) against the
oracle and the committed golden fixture.

Tolerance (BASELINE.md "Parity"; fp32 kernels vs float64 truth): per output
table, normwise relative error <= 1e-5 AND max-abs error <= 1e-5 * max|ref|.
Integer/index outputs (CSR, plan, sampler invariants) are exact.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from bbgr import _lib  # noqa: E402
from bbgr.graph import BipartiteGraph, Csr  # noqa: E402
from bbgr.synthetic import synthetic_credibility, synthetic_edges  # noqa: E402
from oracle import ref_numpy as R  # noqa: E402
from oracle import ref_torch as T  # noqa: E402

DEV = "cuda"
TOL = 1e-5
HERE = os.path.dirname(os.path.abspath(__file__))


def assert_parity(got, ref, what, tol=TOL):
    got = got.detach().double().cpu().numpy() if isinstance(got, torch.Tensor) else got
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    nrm = np.linalg.norm(ref)
    err = np.linalg.norm(got - ref)
    assert err <= tol * max(nrm, 1e-30), f"{what}: normwise rel err {err / max(nrm, 1e-30):.3e}"
    mx = np.abs(ref).max() if ref.size else 0.0
    assert np.abs(got - ref).max() <= tol * max(mx, 1e-30), f"{what}: max-abs err"


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(os.path.join(HERE, "golden", "golden_small.npz")))


def t(a, dtype=torch.float32):
    return torch.as_tensor(np.asarray(a)).to(DEV, dtype)


# ---------------------------------------------------------------------------
# CSR build + plan
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("dup", [0, 50])
def test_csr_build_bit_exact(dup):
    U, I = 500, 300
    e = synthetic_edges(U - 5, I - 5, 6000, 3, items="zipf", duplicates=dup)
    c = Csr(e[0], e[1], U, I, DEV)
    indptr, indices = R.edges_to_user_csr(e, U)
    np.testing.assert_array_equal(c.indptr.cpu().numpy(), indptr)
    np.testing.assert_array_equal(c.indices[: c.nnz].cpu().numpy(), indices)


def test_csr_empty_and_single():
    c = Csr(np.zeros(0, np.int32), np.zeros(0, np.int32), 7, 3, DEV)
    assert c.indptr.cpu().tolist() == [0] * 8
    c = Csr([6], [2], 7, 3, DEV)
    assert c.indptr.cpu().tolist() == [0] * 7 + [1] and c.indices[:1].item() == 2


def test_plan_chunks_cover_long_rows():
    e = synthetic_edges(2000, 100, 40000, 5, items="zipf")
    c = Csr(e[1], e[0], 100, 2000, DEV, long_threshold=64, chunk_edges=128)
    deg = np.bincount(e[1], minlength=100)
    chunks = c.chunks[: 4 * c.n_chunks].view(-1, 4).cpu().numpy()
    covered = np.zeros(100, np.int64)
    for row, b, en, slot in chunks:
        covered[row] += en - b
        assert en - b <= 128
    np.testing.assert_array_equal(covered[deg > 64], deg[deg > 64])
    assert (covered[deg <= 64] == 0).all()
    assert c.n_split == int(((deg > 64) & (deg > 128)).sum())


# ---------------------------------------------------------------------------
# Single fused SpMM vs scipy float64, all weight modes and dims
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("d", [8, 16, 32, 64, 128, 256])
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("thr", [256, 8])
def test_spmm_modes(d, mode, thr):
    from bbgr.propagate import Product, spmm
    rng = np.random.default_rng(d + mode + thr)
    R_, C_ = 400, 350
    e = synthetic_edges(C_ - 3, R_ - 3, 9000, 7, items="zipf", duplicates=20)
    rows, cols = e[1], e[0]                     # item rows (skewed)
    vals = rng.uniform(0.1, 1.0, rows.size).astype(np.float32)
    cs = rng.uniform(0.5, 2.0, C_).astype(np.float32)
    c = Csr(rows, cols, R_, C_, DEV, edge_values=t(vals) if mode == 1 else None,
            long_threshold=thr, chunk_edges=32)
    prod = Product(c, c.values if mode == 1 else None, t(cs) if mode == 2 else None, None, {})
    x = rng.uniform(-1, 1, (C_, d)).astype(np.float32)
    w = vals if mode == 1 else (cs[cols] if mode == 2 else np.ones(rows.size, np.float32))
    Tm = R.csr64(rows, cols, w, (R_, C_)) @ x.astype(np.float64)
    ys = rng.uniform(0.5, 1.5, R_).astype(np.float32)
    add = rng.normal(size=(R_, d)).astype(np.float32)
    adds = rng.uniform(0.5, 1.5, R_).astype(np.float32)
    acc_in = rng.normal(size=(R_, d)).astype(np.float32)
    accs = rng.uniform(0.5, 1.5, R_).astype(np.float32)
    y = torch.empty(R_, d, device=DEV)
    acc = torch.empty(R_, d, device=DEV)
    spmm(prod, t(x), True, y=y, y_scale=t(ys), y_scale_s=0.75, add=t(add), add_scale=t(adds),
         add_scale_s=0.5, acc_in=t(acc_in), acc_out=acc, acc_scale=t(accs), acc_scale_s=1.25,
         gamma=0.25)
    want_y = 0.75 * ys[:, None] * Tm + 0.5 * adds[:, None] * add
    want_acc = 0.25 * (acc_in + 1.25 * accs[:, None] * Tm)
    assert_parity(y, want_y, "y")
    assert_parity(acc, want_acc, "acc")


@pytest.mark.parametrize("d", [8, 16, 32])
def test_narrow_spmm_masks_lists_and_fused_adam(d):
    """Column-shard widths (d/4 lanes per row): src mask, row mask, row list
    (with chunked rows flagged in the mask) and the fused Adam epilogue against
    float64 / the separate Adam on the materialised product."""
    from bbgr.optim import AdamRows
    from bbgr.propagate import Product, spmm
    rng = np.random.default_rng(d)
    R_, C_ = 600, 2500
    e = synthetic_edges(C_, R_, 40000, 5, items="zipf")
    rows, cols = e[1], e[0]
    c = Csr(rows, cols, R_, C_, DEV, long_threshold=32, chunk_edges=128)
    assert c.n_split > 0
    prod = Product(c, None, None, None, {})
    x = rng.uniform(-1, 1, (C_, d)).astype(np.float32)
    src = (rng.random(C_) < 0.2).astype(np.uint8)
    rmask = (rng.random(R_) < 0.3).astype(np.uint8)
    M = R.csr64(rows, cols, np.ones(rows.size, np.float32), (R_, C_))
    full = M @ x.astype(np.float64)
    y = torch.empty(R_, d, device=DEV)
    spmm(prod, t(x), False, y=y)
    assert_parity(y, full, "plain")
    y = torch.zeros(R_, d, device=DEV)
    spmm(prod, t(x), False, y=y, src_mask=t(src, torch.uint8))
    assert_parity(y, M @ (x.astype(np.float64) * src[:, None]), "src mask")
    y = torch.zeros(R_, d, device=DEV)
    spmm(prod, t(x), False, y=y, row_mask=t(rmask, torch.uint8))
    assert_parity(y, full * rmask[:, None], "row mask")
    lst = torch.as_tensor(np.flatnonzero(rmask), dtype=torch.int64, device=DEV)
    y = torch.zeros(R_, d, device=DEV)
    spmm(prod, t(x), False, y=y, row_mask=t(rmask, torch.uint8), row_list=lst)
    assert_parity(y, full * rmask[:, None], "row list")
    p0 = rng.normal(size=(R_, d)).astype(np.float32)
    p1, m1, v1 = t(p0), torch.full((R_, d), 0.01, device=DEV), torch.full((R_, d), 0.02, device=DEV)
    spmm(prod, t(x), False, adam=AdamRows(p1, m1, v1, 3, 1e-3))
    p2, m2, v2 = t(p0), torch.full((R_, d), 0.01, device=DEV), torch.full((R_, d), 0.02, device=DEV)
    g = torch.empty(R_, d, device=DEV)
    spmm(prod, t(x), False, y=g)
    AdamRows(p2, m2, v2, 3, 1e-3).apply(g)
    assert torch.equal(p1, p2) and torch.equal(m1, m2) and torch.equal(v1, v2)


def test_column_shard_forward_equals_full_width_columns():
    """One column shard alone (ColumnShardedTrainer without a process group):
    its forward tables are the full-width trainer's columns [c0, c1)."""
    from bbgr.columns import ColumnShardedTrainer
    from bbgr.trainer import FusedTrainer
    U, I = 2000, 700
    e = synthetic_edges(U, I, 30000, 13, items="zipf")
    rng = np.random.default_rng(13)
    u0 = rng.uniform(-0.5, 0.5, (U, 64)).astype(np.float32)
    i0 = rng.uniform(-0.5, 0.5, (I, 64)).astype(np.float32)
    cred = synthetic_credibility(U, 13)
    full = FusedTrainer(BipartiteGraph(e, U, I, DEV, vertex_order="degree"), "v2_pop", cred=cred,
                        emb_dim=64, num_layers=3, batch_size=256, u0=u0, i0=i0)
    uf, itf = (x.double().cpu().numpy() for x in full.forward())
    for parts in (2, 4, 8):
        for idx in (0, parts - 1):
            sh = ColumnShardedTrainer(e, U, I, "v2_pop", cred=cred, emb_dim=64, num_layers=3,
                                      batch_size=256, u0=u0, i0=i0, column_parts=parts,
                                      column_index=idx, device=DEV)
            su, si = sh.forward()
            c0, c1 = sh.c0, sh.c1
            assert c1 - c0 == 64 // parts
            assert_parity(su, uf[:, c0:c1], f"users {parts}/{idx}")
            assert_parity(si, itf[:, c0:c1], f"items {parts}/{idx}")


@pytest.mark.parametrize("d", [64, 128])
def test_spmm_f32_blueprint_entry_point(d):
    """bbgr_spmm_f32 (SURVEY §8(b)'s flat form): Y = diag(rs) A diag(cs) X and
    acc += a * Y, against float64; a plan with split rows is refused."""
    import ctypes
    from bbgr._lib import call, ld, ptr, stream_handle
    import scipy.sparse as sp
    U, I = 900, 400
    e = synthetic_edges(U, I, 12000, 17, items="zipf")
    c = Csr(e[1], e[0], I, U, DEV, long_threshold=1 << 30)   # no split rows
    assert c.n_split == 0
    rng = np.random.default_rng(d)
    x = rng.normal(size=(U, d)).astype(np.float32)
    rs = rng.uniform(0.5, 1.5, I).astype(np.float32)
    cs = rng.uniform(0.5, 1.5, U).astype(np.float32)
    acc0 = rng.normal(size=(I, d)).astype(np.float32)
    X, RS, CS = t(x), t(rs), t(cs)
    Y = torch.empty(I, d, device=DEV)
    acc = t(acc0)
    call("bbgr_spmm_f32", ctypes.byref(c._struct), ptr(X), ld(X), ptr(Y), ld(Y), d, ptr(RS),
         ptr(CS), ptr(acc), 0.25, stream_handle())
    A = sp.csr_matrix((np.ones(e.shape[1]), (e[1], e[0])), shape=(I, U))
    ref = (rs[:, None].astype(np.float64) * (A @ (cs[:, None].astype(np.float64) * x)))
    assert_parity(Y, ref, "spmm_f32 Y")
    assert_parity(acc, acc0 + 0.25 * ref, "spmm_f32 acc")
    split = Csr(e[1], e[0], I, U, DEV, long_threshold=8, chunk_edges=16)
    assert split.n_split > 0
    with pytest.raises(RuntimeError, match="split rows"):
        call("bbgr_spmm_f32", ctypes.byref(split._struct), ptr(X), ld(X), ptr(Y), ld(Y), d,
             None, None, None, 0.0, stream_handle())


def test_spmm_deterministic():
    from bbgr.propagate import Product, spmm
    e = synthetic_edges(3000, 500, 60000, 9, items="zipf")
    c = Csr(e[1], e[0], 500, 3000, DEV, long_threshold=32, chunk_edges=64)
    prod = Product(c, None, None, None, {})
    x = torch.randn(3000, 64, device=DEV)
    y1, y2 = torch.empty(500, 64, device=DEV), torch.empty(500, 64, device=DEV)
    spmm(prod, x, False, y=y1)
    spmm(prod, x, False, y=y2)
    assert torch.equal(y1, y2)


def test_spmm_unsupported_dim_raises():
    from bbgr.propagate import Product, spmm
    c = Csr([0], [0], 1, 1, DEV)
    with pytest.raises(_lib.BbgrError, match="UNSUPPORTED"):
        spmm(Product(c, None, None, None, {}), torch.zeros(1, 48, device=DEV), False,
             y=torch.zeros(1, 48, device=DEV))


# ---------------------------------------------------------------------------
# Drop-in modules vs golden (forward + autograd backward)
# ---------------------------------------------------------------------------
def _load(model, g):
    with torch.no_grad():
        if hasattr(model, "emb"):
            model.emb.weight.copy_(t(np.concatenate([g["u0"], g["i0"]])))
        else:
            model.user_emb.weight.copy_(t(g["u0"]))
            model.item_emb.weight.copy_(t(g["i0"]))


def test_v2_lightgcn_forward_backward_vs_golden(gold):
    from bbgr.lightgcn_cu_pop import LightGCN, build_message_passing_mats
    U, I, E, DUP, D, K, B = (int(x) for x in gold["meta"])
    M_ui, M_iu = build_message_passing_mats(gold["edges"], U, I, t(gold["cred"]), DEV)
    assert tuple(M_ui.shape) == (U, I) and tuple(M_iu.shape) == (I, U)
    m = LightGCN(U, I, D, K, M_ui, M_iu).to(DEV)
    assert set(m.state_dict()) == {"user_emb.weight", "item_emb.weight"}
    _load(m, gold)
    uf, itf = m.get_user_item_emb()
    assert_parity(uf, gold["gs_uf"], "gs u_final")
    assert_parity(itf, gold["gs_if"], "gs i_final")
    ((uf * t(gold["gU"])).sum() + (itf * t(gold["gI"])).sum()).backward()
    assert_parity(m.user_emb.weight.grad, gold["gs_gu0"], "gs grad u0")
    assert_parity(m.item_emb.weight.grad, gold["gs_gi0"], "gs grad i0")


def test_method_a_forward_vs_golden(gold):
    from bbgr.lightgcn_cu_pop_long_tail_exposure import LightGCN, build_message_passing_mats
    U, I, E, DUP, D, K, B = (int(x) for x in gold["meta"])
    M_ui, M_iu = build_message_passing_mats(gold["edges"], U, I, t(gold["cred"]), DEV)
    m = LightGCN(U, I, D, K, M_ui, M_iu).to(DEV)
    _load(m, gold)
    uf, itf = m.propagate()
    assert_parity(uf, gold["ma_uf"], "method-A u_final")
    assert_parity(itf, gold["ma_if"], "method-A i_final")


def test_cred_lightgcn_jacobi_vs_golden(gold):
    from bbgr.lightgcn_cu import CredLightGCN, build_cred_weighted_mats
    U, I, E, DUP, D, K, B = (int(x) for x in gold["meta"])
    M_ui, M_iu, deg_i = build_cred_weighted_mats(gold["edges"], U, I, gold["cred"], DEV)
    assert tuple(M_ui.shape) == (I, U) and tuple(M_iu.shape) == (U, I)
    np.testing.assert_array_equal(deg_i, np.bincount(gold["edges"][1], minlength=I))
    m = CredLightGCN(U, I, D, K, M_ui, M_iu).to(DEV)
    _load(m, gold)
    uf, itf = m.final_embeddings()
    assert_parity(uf, gold["j_uf"], "J u_final")
    assert_parity(itf, gold["j_if"], "J i_final")
    ((uf * t(gold["gU"])).sum() + (itf * t(gold["gI"])).sum()).backward()
    assert_parity(m.user_emb.weight.grad, gold["j_gu0"], "J grad u0")
    assert_parity(m.item_emb.weight.grad, gold["j_gi0"], "J grad i0")
    # unfused per-layer path gives the same means
    us, is_ = m.propagate_all_layers()
    assert_parity(torch.stack(us).mean(0), gold["j_uf"], "J per-layer mean u")
    assert_parity(torch.stack(is_).mean(0), gold["j_if"], "J per-layer mean i")


def test_plain_lightgcn_sym_vs_golden(gold):
    from bbgr.lightgcn import LightGCN, build_norm_adj
    U, I, E, DUP, D, K, B = (int(x) for x in gold["meta"])
    A = build_norm_adj(gold["edges"], U, I, DEV)
    m = LightGCN(U, I, D, K, A).to(DEV)
    assert set(m.state_dict()) == {"emb.weight"}
    _load(m, gold)
    xf = m.propagate()
    assert_parity(xf, gold["sym_xf"], "sym x_final")
    (xf * t(np.concatenate([gold["gU"], gold["gI"]]))).sum().backward()
    assert_parity(m.emb.weight.grad, gold["sym_gx"], "sym grad")
    uf, itf = m.get_user_item_emb()
    assert uf.shape == (U, D) and itf.shape == (I, D)


def test_torch_sparse_operators_are_accepted(gold):
    """LightGCN fed the reference's own COO tensors (generic explicit-value path)."""
    from bbgr.lightgcn import LightGCN as PlainLightGCN
    from bbgr.lightgcn_cu_pop import LightGCN
    U, I, E, DUP, D, K, B = (int(x) for x in gold["meta"])
    M_ui, M_iu = T.gs_operators(gold["edges"], U, I, gold["cred"], device=DEV)
    m = LightGCN(U, I, D, K, M_ui, M_iu).to(DEV)
    _load(m, gold)
    uf, itf = m.propagate()
    assert_parity(uf, gold["gs_uf"], "coo gs u_final")
    assert_parity(itf, gold["gs_if"], "coo gs i_final")
    ((uf * t(gold["gU"])).sum() + (itf * t(gold["gI"])).sum()).backward()
    assert_parity(m.user_emb.weight.grad, gold["gs_gu0"], "coo gs grad u0")
    A = T.sym_operator(gold["edges"], U, I, device=DEV)
    pm = PlainLightGCN(U, I, D, K, A).to(DEV)
    _load(pm, gold)
    xf = pm.propagate()
    assert_parity(xf, gold["sym_xf"], "coo sym x_final")
    (xf * t(np.concatenate([gold["gU"], gold["gI"]]))).sum().backward()
    assert_parity(pm.emb.weight.grad, gold["sym_gx"], "coo sym grad")


def test_operator_to_torch_sparse_matches_reference_values(gold):
    from bbgr.lightgcn_cu_pop import build_message_passing_mats
    U, I = int(gold["meta"][0]), int(gold["meta"][1])
    M_ui, M_iu = build_message_passing_mats(gold["edges"], U, I, t(gold["cred"]), DEV)
    R_ui, R_iu = R.gs_mats(gold["edges"], U, I, gold["cred"])
    assert_parity(M_ui.to_torch_sparse().to_dense(), R_ui.toarray(), "M_ui values")
    assert_parity(M_iu.to_torch_sparse().to_dense(), R_iu.toarray(), "M_iu values")
    x = np.random.default_rng(0).normal(size=(U, 64)).astype(np.float32)
    assert_parity(M_iu @ t(x), R_iu @ x.astype(np.float64), "M_iu @ x")


# ---------------------------------------------------------------------------
# BPR, Adam
# ---------------------------------------------------------------------------
def test_bpr_loss_and_grads_vs_golden(gold):
    from bbgr.bpr import bpr_loss
    uf = t(gold["gs_uf"]).requires_grad_()
    itf = t(gold["gs_if"]).requires_grad_()
    ue = t(gold["u0"]).requires_grad_()
    ie = t(gold["i0"]).requires_grad_()
    loss = bpr_loss(t(gold["users"], torch.int64), t(gold["pos"], torch.int64),
                    t(gold["neg"], torch.int64), uf, itf, ue, ie, 1e-4, pop=t(gold["pop"]),
                    lambda_fair=0.05)
    assert abs(float(loss.detach()) - float(gold["bpr_loss"])) <= TOL * abs(float(gold["bpr_loss"]))
    loss.backward()
    assert_parity(uf.grad, gold["bpr_g_uf"], "bpr g_uf")
    assert_parity(itf.grad, gold["bpr_g_if"], "bpr g_if")
    assert_parity(ue.grad, gold["bpr_g_ue"], "bpr g_ue")
    assert_parity(ie.grad, gold["bpr_g_ie"], "bpr g_ie")


def test_bpr_ln2_at_zero_embeddings():
    from bbgr.bpr import bpr_loss_value
    z = torch.zeros(10, 64, device=DEV)
    idx = torch.arange(8, device=DEV)
    loss = bpr_loss_value(idx, idx, idx + 1, z, z, z, z, 1e-4)
    assert abs(float(loss) - np.log(2.0)) < 1e-6


def test_fused_adam_vs_golden_and_torch(gold):
    from bbgr.optim import FusedAdam, adam_step
    p = t(gold["u0"]).clone()
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    adam_step(p, t(gold["gU"]), m, v, 1, 1e-3)
    assert_parity(p, gold["adam_p1"], "adam step 1", tol=1e-6)
    a = torch.nn.Parameter(t(gold["u0"]).clone())
    b = torch.nn.Parameter(t(gold["u0"]).clone())
    oa, ob = FusedAdam([a], lr=1e-3), torch.optim.Adam([b], lr=1e-3)
    rng = np.random.default_rng(1)
    for _ in range(5):
        g = t(rng.normal(size=a.shape))
        a.grad, b.grad = g.clone(), g.clone()
        oa.step()
        ob.step()
    assert_parity(a.detach(), b.detach().double().cpu().numpy(), "FusedAdam vs torch Adam",
                  tol=1e-6)


# ---------------------------------------------------------------------------
# Samplers
# ---------------------------------------------------------------------------
def _graph(U=2000, I=800, E=30000, seed=3):
    e = synthetic_edges(U, I, E, seed, items="zipf")
    return e, BipartiteGraph(e, U, I, DEV)


def test_sampler_invariants_and_determinism():
    from bbgr.sampler import PopMixSampler
    e, g = _graph()
    indptr, indices = R.edges_to_user_csr(e, 2000)
    s = PopMixSampler(g.user_csr, g.item_csr, 800, mix_pop=0.7, gamma=0.75, max_tries=50, seed=42)
    users = torch.arange(2000, device=DEV)
    pos, neg = s.sample(users, counter=5)
    p, n = pos.cpu().numpy(), neg.cpu().numpy()
    for u in range(2000):
        assert R.user_has_item(indptr, indices, u, p[u])
        assert not R.user_has_item(indptr, indices, u, n[u])
    pos2, neg2 = s.sample(users, counter=5)
    assert torch.equal(pos, pos2) and torch.equal(neg, neg2)
    pos3, neg3 = s.sample(users, counter=6)
    assert not torch.equal(neg, neg3)
    assert int(s.fail_count.item()) == 0


def test_sampler_popularity_distribution_chi2():
    """mix_pop = 1 and a tiny graph (rejections rare): negatives follow pop_prob."""
    from bbgr.sampler import PopMixSampler
    U, I = 4000, 50
    e = synthetic_edges(U, I, U, 8, items="zipf")        # one edge per user
    g = BipartiteGraph(e, U, I, DEV)
    s = PopMixSampler(g.user_csr, g.item_csr, I, mix_pop=1.0, gamma=0.75, max_tries=50, seed=1)
    counts = np.zeros(I)
    users = torch.arange(U, device=DEV)
    for c in range(50):
        _, neg = s.sample(users, counter=c)
        counts += np.bincount(neg.cpu().numpy(), minlength=I)
    pp = R.pop_prob(e, I)
    # exact expectation with one rejected item per user: renormalise per user
    indptr, indices = R.edges_to_user_csr(e, U)
    exp = np.zeros(I)
    for u in range(U):
        q = pp.copy()
        q[indices[indptr[u]:indptr[u + 1]]] = 0
        exp += q / q.sum()
    exp *= 50
    chi2 = ((counts - exp) ** 2 / exp).sum()
    assert chi2 < 2.0 * I, chi2          # dof = 49; generous bound


def test_pop_cdf_matches_oracle_on_many_blocks():
    """The pop-mix CDF (bbgr_pop_cdf) over ~1200 workgroups equals the
    reference's normalised cumsum of pop_prob (Version-2:805-810), every
    build (a race in an in-place normalisation once left blocks unscaled)."""
    from bbgr.sampler import PopMixSampler
    U, I = 20000, 300_000
    e = synthetic_edges(U, I, 400_000, 21, items="zipf")
    g = BipartiteGraph(e, U, I, DEV)
    pp = R.pop_prob(e, I)
    want = np.cumsum(pp) / np.cumsum(pp)[-1]
    for _ in range(5):
        s = PopMixSampler(g.user_csr, g.item_csr, I, mix_pop=0.7, gamma=0.75, seed=1)
        got = s.cdf.cpu().numpy()
        assert got[-1] == 1.0 and np.all(np.diff(got) >= 0)
        np.testing.assert_allclose(got, want, rtol=1e-9, atol=0)


def test_sampler_full_row_user_flags_failure():
    from bbgr.sampler import PopMixSampler
    e = np.array([[0, 0, 0, 1], [0, 1, 2, 0]], np.int32)   # user 0 holds every item
    g = BipartiteGraph(e, 2, 3, DEV)
    s = PopMixSampler(g.user_csr, g.item_csr, 3, mix_pop=0.0, gamma=None, max_tries=5)
    pos, neg = s.sample(torch.tensor([0, 1], device=DEV))
    assert neg[0].item() == -1 and int(s.fail_count.item()) == 1
    assert neg[1].item() in (1, 2)


def test_step_with_a_user_holding_every_item():
    """The reference's negative loop never ends for a user who holds every item
    (Version-2:364-376). Here the sampler gives up (neg = -1, fail_count += 1),
    the BPR kernel drops that triple (no loss, no gradient) and the batch mean
    still divides by B: loss = (B-1)/B x the oracle mean over the kept triples."""
    from bbgr.trainer import FusedTrainer
    rng = np.random.default_rng(4)
    U, I, d, K = 60, 20, 64, 2
    rows = [np.zeros(I, np.int32)]                     # user 0: every item
    cols = [np.arange(I, dtype=np.int32)]
    for u in range(1, U):
        it = rng.choice(I, 3, replace=False).astype(np.int32)
        rows.append(np.full(3, u, np.int32))
        cols.append(it)
    e = np.vstack([np.concatenate(rows), np.concatenate(cols)])
    u0 = rng.uniform(-0.5, 0.5, (U, d)).astype(np.float32)
    i0 = rng.uniform(-0.5, 0.5, (I, d)).astype(np.float32)
    g = BipartiteGraph(e, U, I, DEV)
    tr = FusedTrainer(g, "cu_message", emb_dim=d, num_layers=K, batch_size=U, u0=u0, i0=i0,
                      neg_max_tries=5, frontier=False)
    loss = float(tr.step())
    users, pos, neg = (x.cpu().numpy() for x in tr.batch())
    assert (neg == -1).sum() == 1 and users[neg == -1][0] == 0
    assert int(tr.sampler.fail_count.item()) == 1
    keep = neg >= 0
    M_ui, M_iu = R.gs_mats(e, U, I)
    uf, itf, _, _ = R.propagate_gs(M_ui, M_iu, u0, i0, K)
    want, _ = R.bpr_loss(uf, itf, u0, i0, users[keep], pos[keep], neg[keep], 1e-4)
    assert abs(loss - want * keep.sum() / U) <= 1e-5 * want


def test_shuffle_and_nonempty_rows():
    from bbgr.sampler import nonempty_rows, shuffle
    e = np.array([[0, 2, 2, 5], [0, 1, 2, 0]], np.int32)
    g = BipartiteGraph(e, 7, 3, DEV)
    assert nonempty_rows(g.user_csr).cpu().tolist() == [0, 2, 5]
    v = torch.arange(100000, device=DEV)
    p1 = shuffle(v, 42, 1)
    assert torch.equal(torch.sort(p1).values, v) and not torch.equal(p1, v)
    assert torch.equal(p1, shuffle(v, 42, 1)) and not torch.equal(p1, shuffle(v, 42, 2))


# ---------------------------------------------------------------------------
# Fused training step vs the float64 oracle step on identical triples
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("variant", ["v2_pop", "cu_fair", "method_a"])
def test_fused_trainer_step_vs_oracle(gold, variant):
    from bbgr.trainer import FusedTrainer
    U, I, E, DUP, D, K, B = (int(x) for x in gold["meta"])
    e, cred = gold["edges"], gold["cred"]
    g = BipartiteGraph(e, U, I, DEV)
    lam = 0.05 if variant == "cu_fair" else 0.0
    tr = FusedTrainer(g, variant, cred=cred, emb_dim=D, num_layers=K, batch_size=B,
                      lambda_fair=lam, u0=gold["u0"], i0=gold["i0"], fuse_adam=False,
                      frontier=True)
    deg_u = np.bincount(e[0], minlength=U)
    uu = np.unique(gold["users"])
    users = t(uu[deg_u[uu] > 0], torch.int64)       # train users have >= 1 positive
    loss = tr.step(users)
    pos, neg = tr.pos[: users.numel()].cpu().numpy(), tr.neg[: users.numel()].cpu().numpy()
    uu = users.cpu().numpy()
    # oracle step on the same triples
    if variant == "cu_fair":
        A, Bm, deg_i = R.j_mats(e, U, I, cred)
        uf, itf, _, _ = R.propagate_j(A, Bm, gold["u0"], gold["i0"], K)
        pop = deg_i / max(deg_i.max(), 1.0)
    else:
        A, Bm = R.gs_mats(e, U, I, cred, method_a=(variant == "method_a"))
        uf, itf, _, _ = R.propagate_gs(A, Bm, gold["u0"], gold["i0"], K)
        pop = None
    want_loss, gr = R.bpr_loss(uf, itf, gold["u0"], gold["i0"], uu, pos, neg, 1e-4, pop, lam)
    if variant == "cu_fair":
        gu0, gi0 = R.backward_j(A, Bm, gr["g_uf"], gr["g_if"], K)
    else:
        gu0, gi0 = R.backward_gs(A, Bm, gr["g_uf"], gr["g_if"], K)
    gu0, gi0 = gu0 + gr["g_ue"], gi0 + gr["g_ie"]
    assert abs(float(loss) - want_loss) <= TOL * want_loss
    # the weight gradients the step fed to Adam: the parity claim (1e-5)
    assert_parity(tr.g_u0, gu0, "grad u0 (propagated + ego L2)")
    assert_parity(tr.g_i0, gi0, "grad i0 (propagated + ego L2)")
    # Adam's first step is ~ -lr*sign(g): elements with |g| ~ eps amplify ulp-level
    # gradient differences, so the update itself is compared normwise only.
    z = np.zeros_like
    pu, _, _ = R.adam_step(gold["u0"], gu0, z(gu0), z(gu0), 1)
    pi, _, _ = R.adam_step(gold["i0"], gi0, z(gi0), z(gi0), 1)
    for got, want, name in ((tr.user_w - t(gold["u0"]), pu - gold["u0"], "user update"),
                            (tr.item_w - t(gold["i0"]), pi - gold["i0"], "item update")):
        got = got.double().cpu().numpy()
        assert np.linalg.norm(got - want) <= 1e-4 * np.linalg.norm(want), name
    assert tr.g_uf.abs().sum().item() == 0 and tr.g_if.abs().sum().item() == 0


@pytest.mark.parametrize("K,d,frontier", [(0, 64, True), (1, 64, True), (4, 64, True),
                                         (2, 128, True), (3, 256, True), (3, 128, False)])
def test_fused_trainer_shapes_vs_oracle(K, d, frontier):
    """The GS training step (fused Adam, frontier masks) at other depths and
    widths: loss at 1e-5 and the Adam update normwise vs the float64 oracle."""
    from bbgr.trainer import FusedTrainer
    U, I = 1500, 700
    e = synthetic_edges(U, I, 20000, 31 + K + d, items="zipf", duplicates=30)
    cred = synthetic_credibility(U, 5)
    rng = np.random.default_rng(K + d)
    u0 = rng.uniform(-0.3, 0.3, (U, d)).astype(np.float32)
    i0 = rng.uniform(-0.3, 0.3, (I, d)).astype(np.float32)
    g = BipartiteGraph(e, U, I, DEV)
    tr = FusedTrainer(g, "v2_pop", cred=cred, emb_dim=d, num_layers=K, batch_size=300,
                      u0=u0, i0=i0, frontier=frontier)
    users = tr.next_users()
    loss = float(tr.step(users))
    B = users.numel()
    uu = users.cpu().numpy()
    pos, neg = tr.pos[:B].cpu().numpy(), tr.neg[:B].cpu().numpy()
    A, Bm = R.gs_mats(e, U, I, cred)
    uf, itf, _, _ = R.propagate_gs(A, Bm, u0, i0, K)
    want, gr = R.bpr_loss(uf, itf, u0, i0, uu, pos, neg, 1e-4)
    assert abs(loss - want) <= TOL * want, (loss, want)
    gu0, gi0 = R.backward_gs(A, Bm, gr["g_uf"], gr["g_if"], K)
    gu0, gi0 = gu0 + gr["g_ue"], gi0 + gr["g_ie"]
    z = np.zeros_like
    pu, _, _ = R.adam_step(u0, gu0, z(gu0), z(gu0), 1)
    pi, _, _ = R.adam_step(i0, gi0, z(gi0), z(gi0), 1)
    for got, want_, name in ((tr.user_w - t(u0), pu - u0, "user update"),
                             (tr.item_w - t(i0), pi - i0, "item update")):
        got = got.double().cpu().numpy()
        assert np.linalg.norm(got - want_) <= 1e-4 * np.linalg.norm(want_), name
    assert tr.g_uf.abs().sum().item() == 0 and tr.g_if.abs().sum().item() == 0


def test_dropin_training_step_matches_reference_torch_step(gold):
    """One step of the drop-in module + torch Adam == the fp32 torch restatement."""
    from bbgr.lightgcn_cu_pop import LightGCN, build_message_passing_mats
    U, I, E, DUP, D, K, B = (int(x) for x in gold["meta"])
    e, cred = gold["edges"], gold["cred"]
    users = torch.as_tensor(np.unique(gold["users"]))
    pos = torch.as_tensor(gold["pos"][: users.numel()])
    neg = torch.as_tensor(gold["neg"][: users.numel()])
    M_ui, M_iu = build_message_passing_mats(e, U, I, t(cred), DEV)
    m = LightGCN(U, I, D, K, M_ui, M_iu).to(DEV)
    _load(m, gold)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    ue, ie = m.get_user_item_emb()
    loss = m.bpr_loss(users.to(DEV), pos.to(DEV), neg.to(DEV), ue, ie, 1e-4)
    opt.zero_grad()
    loss.backward()
    opt.step()
    Tui, Tiu = T.gs_operators(e, U, I, cred)
    ref = T.GSModel(U, I, D, K, Tui, Tiu, gold["u0"], gold["i0"])
    ropt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    rloss = T.train_step(ref, ropt, users, pos, neg, 1e-4)
    assert abs(float(loss) - rloss) <= 1e-5 * rloss
    du = (m.user_emb.weight.detach().cpu() - torch.as_tensor(gold["u0"])).double().numpy()
    rdu = (ref.user_emb.weight.detach() - torch.as_tensor(gold["u0"])).double().numpy()
    # Adam step 1 ~ -lr*sign(g): normwise comparison (see the trainer test)
    assert np.linalg.norm(du - rdu) <= 1e-4 * np.linalg.norm(rdu)


# ---------------------------------------------------------------------------
# Larger sizes: C2 parity, size-independent properties
# ---------------------------------------------------------------------------
def test_c2_forward_parity_and_adjoint():
    from bbgr.synthetic import CONFIGS, config_edges
    from bbgr.propagate import ORDER_GS, OperatorPair, backward, forward
    c = CONFIGS["C2"]
    U, I, d, K = c["num_users"], c["num_items"], c["emb_dim"], c["num_layers"]
    e = config_edges("C2")
    cred = synthetic_credibility(U, 2)
    g = BipartiteGraph(e, U, I, DEV)
    pair = OperatorPair.factored(g, g.scales(_lib.OP_GS, t(cred)))
    rng = np.random.default_rng(2)
    u0 = rng.uniform(-1, 1, (U, d)).astype(np.float32)
    i0 = rng.uniform(-1, 1, (I, d)).astype(np.float32)
    uf, itf = forward(pair, t(u0), t(i0), K, ORDER_GS)
    M_ui, M_iu = R.gs_mats(e, U, I, cred)
    ruf, ritf, _, _ = R.propagate_gs(M_ui, M_iu, u0, i0, K)
    assert_parity(uf, ruf, "C2 u_final")
    assert_parity(itf, ritf, "C2 i_final")
    gU = rng.normal(size=(U, d)).astype(np.float32)
    gI = rng.normal(size=(I, d)).astype(np.float32)
    gu0, gi0 = backward(pair, t(gU), t(gI), K, ORDER_GS)
    # the backward against the float64 autograd adjoint of the reference chain
    # (oracle backward_gs: Version-2:482-489 differentiated, V2:862)
    rgu0, rgi0 = R.backward_gs(M_ui, M_iu, gU, gI, K)
    assert_parity(gu0, rgu0, "C2 grad u0")
    assert_parity(gi0, rgi0, "C2 grad i0")
    lhs = (uf.double() * t(gU).double()).sum() + (itf.double() * t(gI).double()).sum()
    rhs = (t(u0).double() * gu0.double()).sum() + (t(i0).double() * gi0.double()).sum()
    assert abs(float(lhs - rhs)) <= 1e-5 * abs(float(lhs))


@pytest.mark.slow
def test_c4_size_adjoint_and_linearity():
    """Full BASELINE C4 size: <F(x), g> == <x, F^T(g)> and F(2x) == 2 F(x)."""
    from bbgr.synthetic import CONFIGS, config_edges
    from bbgr.propagate import ORDER_GS, OperatorPair, backward, forward
    c = CONFIGS["C4"]
    U, I, d, K = c["num_users"], c["num_items"], c["emb_dim"], c["num_layers"]
    e = config_edges("C4")
    g = BipartiteGraph(e, U, I, DEV)
    del e
    pair = OperatorPair.factored(g, g.scales(_lib.OP_GS, None))
    gen = torch.Generator(device=DEV).manual_seed(0)
    u0 = torch.rand(U, d, device=DEV, generator=gen) * 2 - 1
    i0 = torch.rand(I, d, device=DEV, generator=gen) * 2 - 1
    uf, itf = forward(pair, u0, i0, K, ORDER_GS)
    uf2, itf2 = forward(pair, 2 * u0, 2 * i0, K, ORDER_GS)
    assert torch.equal(uf2, 2 * uf) and torch.equal(itf2, 2 * itf)   # exact: power-of-2 scale
    gU = torch.randn(U, d, device=DEV, generator=gen)
    gI = torch.randn(I, d, device=DEV, generator=gen)
    gu0, gi0 = backward(pair, gU, gI, K, ORDER_GS)
    lhs = (uf.double() * gU.double()).sum() + (itf.double() * gI.double()).sum()
    rhs = (u0.double() * gu0.double()).sum() + (i0.double() * gi0.double()).sum()
    assert abs(float(lhs - rhs)) <= 1e-5 * float(
        (uf.double().abs() * gU.double().abs()).sum() + (itf.double().abs() * gI.double().abs()).sum())


# ---------------------------------------------------------------------------
# Frontier masks (exact sparsity)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("thr", [256, 8])
def test_spmm_src_and_row_masks(thr):
    from bbgr.propagate import Product, spmm
    rng = np.random.default_rng(thr)
    R_, C_, d = 400, 350, 64
    e = synthetic_edges(C_, R_, 9000, 4, items="zipf")
    rows, cols = e[1], e[0]
    c = Csr(rows, cols, R_, C_, DEV, long_threshold=thr, chunk_edges=32)
    prod = Product(c, None, None, None, {})
    x = rng.uniform(-1, 1, (C_, d)).astype(np.float32)
    smask = (rng.random(C_) < 0.1).astype(np.uint8)
    rmask = (rng.random(R_) < 0.3).astype(np.uint8)
    y = torch.full((R_, d), 7.0, device=DEV)
    xm = x * smask[:, None]          # the dense equivalent: x is zero off the mask
    spmm(prod, t(xm), False, y=y, src_mask=t(smask, torch.uint8))
    want = R.csr64(rows, cols, np.ones(rows.size), (R_, C_)) @ xm.astype(np.float64)
    assert_parity(y, want, "src-masked y")
    y2 = torch.full((R_, d), 7.0, device=DEV)
    spmm(prod, t(x), False, y=y2, row_mask=t(rmask, torch.uint8))
    full = R.csr64(rows, cols, np.ones(rows.size), (R_, C_)) @ x.astype(np.float64)
    got = y2.cpu().numpy()
    assert_parity(got[rmask == 1], full[rmask == 1], "row-masked y")
    assert (got[rmask == 0] == 7.0).all()          # unflagged rows untouched


@pytest.mark.parametrize("variant", ["v2_pop", "cu_fair"])
def test_frontier_step_matches_dense_step(variant):
    """Frontier-masked training step == dense step (C2 graph, long rows split)."""
    from bbgr.synthetic import CONFIGS, config_edges
    from bbgr.trainer import FusedTrainer
    c = CONFIGS["C2"]
    U, I = c["num_users"], c["num_items"]
    e = config_edges("C2")
    cred = synthetic_credibility(U, 2)
    g = BipartiteGraph(e, U, I, DEV)
    rng = np.random.default_rng(0)
    u0 = rng.uniform(-0.05, 0.05, (U, 64)).astype(np.float32)
    i0 = rng.uniform(-0.05, 0.05, (I, 64)).astype(np.float32)
    kw = dict(cred=cred, emb_dim=64, num_layers=3, batch_size=4096, u0=u0, i0=i0,
              lambda_fair=0.05 if variant == "cu_fair" else 0.0, fuse_adam=False)
    dense = FusedTrainer(g, variant, frontier=False, **kw)
    front = FusedTrainer(g, variant, frontier=True, **kw)
    for _ in range(3):
        users = dense.next_users()
        front.next_users()
        ld_, lf = float(dense.step(users)), float(front.step(users))
        assert torch.equal(dense.pos, front.pos) and torch.equal(dense.neg, front.neg)
        assert abs(ld_ - lf) <= 1e-6 * abs(ld_)
        for a, b, what in ((dense.g_u0, front.g_u0, "grad u0"), (dense.g_i0, front.g_i0, "grad i0")):
            err = (a.double() - b.double()).norm() / a.double().norm()
            assert err <= 1e-6, (what, float(err))
    # masks are left clean for the next step
    assert int(front.mask_u.sum()) == 0 and int(front.mask_i.sum()) == 0


def test_host_length_item_list_is_bitwise_the_device_count(monkeypatch):
    """The trainer's frontier-list launches (last forward item layer, first
    backward item product) take the list at its published host length
    (propagate.ListLength: a grid sized to the list) instead of the capacity
    with the device count: same rows, same arithmetic — losses and weights
    bitwise equal over steps, the published length the device count."""
    from bbgr import propagate as PP
    from bbgr.synthetic import CONFIGS, config_edges
    from bbgr.trainer import FusedTrainer
    c = CONFIGS["C2"]
    U, I = c["num_users"], c["num_items"]
    g = BipartiteGraph(config_edges("C2"), U, I, DEV, vertex_order="degree")
    kw = dict(cred=synthetic_credibility(U, 2), emb_dim=64, num_layers=3, batch_size=4096,
              frontier=True)
    host = FusedTrainer(g, "v2_pop", **kw)
    seen = []
    real = PP.ListLength.length

    def spy(self):
        n = real(self)
        seen.append((n, int(self.count.item()) if n is not None else None))
        return n
    monkeypatch.setattr(PP.ListLength, "length", spy)
    lh = [float(host.step()) for _ in range(3)]
    assert seen and all(n is not None and n == cnt and n > 0 for n, cnt in seen)
    monkeypatch.setattr(PP.ListLength, "length", lambda self: None)   # device count
    dev = FusedTrainer(g, "v2_pop", **kw)
    ld_ = [float(dev.step()) for _ in range(3)]
    assert lh == ld_
    for a, b in ((host.user_w, dev.user_w), (host.item_w, dev.item_w),
                 (host.m_i, dev.m_i), (host.v_u, dev.v_u)):
        assert torch.equal(a, b)


@pytest.mark.parametrize("variant,K", [("v2_pop", 3), ("method_a", 2), ("v2_pop", 1),
                                       ("cu_fair", 3), ("cu_fair", 2), ("plain", 3)])
def test_fused_adam_step_matches_unfused(variant, K):
    """Adam fused into the last backward SpMM (users) and read from the sparse
    BPR table with grad_scale (items) == the separate gradient + Adam path:
    bitwise on rows outside the batch, to fp32 rounding on batch rows (the
    ego-L2 term enters as gl*(gU + a/gl*e0) instead of gl*gU + a*e0)."""
    from bbgr.synthetic import CONFIGS, config_edges
    from bbgr.trainer import FusedTrainer
    c = CONFIGS["C2"]
    U, I = c["num_users"], c["num_items"]
    e = config_edges("C2")
    g = BipartiteGraph(e, U, I, DEV)
    rng = np.random.default_rng(1)
    u0 = rng.uniform(-0.05, 0.05, (U, 64)).astype(np.float32)
    i0 = rng.uniform(-0.05, 0.05, (I, 64)).astype(np.float32)
    kw = dict(cred=synthetic_credibility(U, 2), emb_dim=64, num_layers=K, batch_size=4096,
              u0=u0, i0=i0, frontier=True)
    sep = FusedTrainer(g, variant, fuse_adam=False, **kw)
    fus = FusedTrainer(g, variant, fuse_adam=True, **kw)
    assert fus.fuse_adam and not sep.fuse_adam   # Jacobi: both Adams fused (K >= 2)
    for step in range(3):
        users = sep.next_users()
        fus.next_users()
        ls, lf = float(sep.step(users)), float(fus.step(users))
        assert torch.equal(sep.pos, fus.pos) and torch.equal(sep.neg, fus.neg)
        assert abs(ls - lf) <= 1e-6 * abs(ls)
        if step == 0 and K > 1:   # K == 1: masked last product + separate Adam
            B = users.numel()
            for a, b, rows, n, what in (
                    (sep.user_w, fus.user_w, users, U, "user"),
                    (sep.item_w, fus.item_w, torch.cat([sep.pos[:B], sep.neg[:B]]), I, "item")):
                off = torch.ones(n, dtype=torch.bool, device=DEV)
                off[rows] = False
                assert torch.equal(a[off], b[off]), what      # bitwise off the batch
    for a, b, init, what in ((sep.user_w, fus.user_w, u0, "user"),
                             (sep.item_w, fus.item_w, i0, "item")):
        err = (a.double() - b.double()).norm() / (a.double() - t(init).double()).norm()
        assert err <= 1e-4, (what, float(err))
    for m_s, m_f in ((sep.m_u, fus.m_u), (sep.v_u, fus.v_u), (sep.m_i, fus.m_i)):
        assert (m_s.double() - m_f.double()).norm() <= 1e-4 * m_s.double().norm()
    assert fus.g_uf.abs().sum().item() == 0 and fus.g_if.abs().sum().item() == 0


def test_graph_from_memmaps_matches_array(tmp_path):
    from bbgr import ingest
    e = synthetic_edges(500, 300, 6000, 12, items="zipf")
    np.save(tmp_path / "train_edges.npy", e)
    for name, arr in (("u2i_src.mmap", e[0]), ("u2i_dst.mmap", e[1])):
        m = np.memmap(tmp_path / name, dtype=np.int32, mode="w+", shape=arr.shape)
        m[:] = arr
        m.flush()
    g1 = BipartiteGraph(e, 500, 300, DEV)
    g2 = BipartiteGraph(ingest.load_edges_npy(tmp_path / "train_edges.npy"), 500, 300, DEV)
    g3 = BipartiteGraph(ingest.load_u2i_memmap(tmp_path), 500, 300, DEV)
    for g in (g2, g3):
        assert torch.equal(g.user_csr.indptr, g1.user_csr.indptr)
        assert torch.equal(g.item_csr.indices, g1.item_csr.indices)


@pytest.mark.parametrize("n,hi", [(1, 5), (7, 3), (16384, 1_000_000), (16384, 40), (300, 300)])
def test_first_slot_kernel_is_the_first_occurrence(n, hi):
    """bbgr_first_slot (the C++ operators' ego-row slots): slot[b] is the
    smallest b' with ids[b'] == ids[b], as bpr._first_slot's sort computes
    it; ids outside [0, hi) keep their own slot; the scratch is left all
    INT32_MAX for the next call."""
    import ctypes
    from bbgr import _lib, bpr
    g = torch.Generator().manual_seed(n + hi)
    ids = torch.randint(-1, hi + 1, (n,), generator=g)
    valid = (ids >= 0) & (ids < hi)
    first_of = {}
    for b, v in enumerate(ids.tolist()):
        if 0 <= v < hi:
            first_of.setdefault(v, b)
    want = torch.tensor([first_of.get(v, b) for b, v in enumerate(ids.tolist())])
    # (bpr._first_slot's sort gives the same on the valid entries)
    vb = valid.nonzero().flatten()
    assert torch.equal(vb[bpr._first_slot(ids[valid])], want[valid])
    first = torch.full((hi,), 0x7fffffff, dtype=torch.int32, device=DEV)
    slot = torch.empty(n, dtype=torch.int64, device=DEV)
    idd = ids.to(DEV)
    for _ in range(2):   # reusable scratch
        _lib.call("bbgr_first_slot", n, _lib.ptr(idd), hi, _lib.ptr(first), _lib.ptr(slot),
                  _lib.stream_handle())
        torch.cuda.synchronize()
        got = slot.cpu()
        assert torch.equal(got[valid], want[valid])
        assert torch.equal(got[~valid], torch.arange(n)[~valid])
        assert bool((first == 0x7fffffff).all())


@pytest.mark.parametrize("B,U,I,d", [(1, 3, 2, 64), (8192, 50_000, 20_000, 64), (4096, 50, 30, 64),
                                     (300, 300, 7, 128), (512, 900, 40, 256)])
def test_ego_rows_kernel_is_the_atomic_formulation(B, U, I, d):
    """bbgr_ego_rows (first-slot counts, then each slot's y added n times from
    +0.0) is bitwise the bbgr_bpr ego rows it replaced (float atomics of the
    identical addends, bpr.ego_grad_rows): Zipf-hot items repeated hundreds of
    times, repeated users, invalid triples; the counts scratch is zero again."""
    from bbgr import _lib
    from bbgr import bpr
    g = torch.Generator().manual_seed(B + U + I + d)
    users = torch.randint(0, U, (B,), generator=g)
    zipf = torch.distributions.Categorical(1.0 / torch.arange(1, I + 1, dtype=torch.float64) ** 1.1)
    pos, neg = zipf.sample((B,)), zipf.sample((B,))
    if B > 1:
        users[::7] = users[0]
        users[::97], neg[::89] = -1, I
    du, dp, dn = (x.to(DEV) for x in (users, pos, neg))
    ue = torch.randn(U, d, generator=g).to(DEV)
    ie = torch.randn(I, d, generator=g).to(DEV)
    dl = torch.tensor(0.37, device=DEV)
    want_u, want_i, iu, ii = bpr.ego_grad_rows(dl, du, dp, dn, ue, ie, 1e-2)
    fu = torch.full((U,), 0x7fffffff, dtype=torch.int32, device=DEV)
    fi = torch.full((I,), 0x7fffffff, dtype=torch.int32, device=DEV)
    out = torch.empty(6 * B, dtype=torch.int64, device=DEV)
    P = _lib.ptr
    _lib.call("bbgr_ego_slots", B, P(du), P(dp), P(dn), U, I, P(fu), P(fi), P(out), P(out[B:]),
              P(out[3 * B:]), P(out[4 * B:]), P(out[5 * B:]), _lib.stream_handle())
    cnt = torch.zeros(3 * B, dtype=torch.int32, device=DEV)
    got = torch.full((3 * B, d), 7.0, device=DEV)
    for _ in range(2):   # the counts come back zero: reusable
        _lib.call("bbgr_ego_rows", B, d, P(out[3 * B:]), P(out[4 * B:]), P(out[5 * B:]), P(out),
                  P(out[B:]), P(ue), d, P(ie), d, P(dl), 1e-2, P(cnt), P(got), d, P(got[B:]), d,
                  1.0, None, _lib.stream_handle())
        torch.cuda.synchronize()
        assert torch.equal(got[:B], want_u) and torch.equal(got[B:], want_i)
        assert int(cnt.abs().sum()) == 0
    # scale: the rows times scale in one rounding (the in-backward Adam's K + 1)
    for sc in (3.0, 4.0):
        _lib.call("bbgr_ego_rows", B, d, P(out[3 * B:]), P(out[4 * B:]), P(out[5 * B:]), P(out),
                  P(out[B:]), P(ue), d, P(ie), d, P(dl), 1e-2, P(cnt), P(got), d, P(got[B:]), d,
                  sc, None, _lib.stream_handle())
        torch.cuda.synchronize()
        assert torch.equal(got[:B], want_u * sc) and torch.equal(got[B:], want_i * sc)
        assert int(cnt.abs().sum()) == 0
    if B > 1000:   # the case really repeats rows
        assert int(torch.bincount(torch.cat([pos, neg])).max()) > 100


@pytest.mark.parametrize("B,U,d,invalid_first", [(1, 3, 64, False), (8192, 5_000_000, 64, False),
                                                 (8192, 50_000, 64, True), (4096, 50, 128, True),
                                                 (300, 300, 256, True), (513, 7, 64, False)])
def test_rows_add_slots_is_the_sorted_scatter(B, U, d, invalid_first):
    """bbgr_rows_add_slots (first slots and counts from bbgr_ego_slots /
    bbgr_ego_rows' counts_u_out) is bitwise bbgr_scatter_add_rows over the
    clamped user ids when invalid triples carry zero rows: distinct users,
    users repeated hundreds of times, invalid triples — also one holding the
    first occurrence of a valid user's clamped id (its slot then leads)."""
    from bbgr import _lib
    from bbgr.scatter import index_add_rows
    g = torch.Generator().manual_seed(B + U + d)
    I = 40
    users = torch.randint(0, U, (B,), generator=g) if U < 5_000_000 else torch.randperm(U, generator=g)[:B]
    pos, neg = torch.randint(0, I, (B,), generator=g), torch.randint(0, I, (B,), generator=g)
    if invalid_first:
        users[0], users[1] = -1, 0     # clamp(-1) = 0: the invalid slot 0 leads user 0
        users[5::11] = U + 3            # clamps to U - 1
        neg[7::13] = I                 # an invalid item: the user's slot is invalid too
    du, dp, dn = (x.to(DEV) for x in (users, pos, neg))
    fu = torch.full((U,), 0x7fffffff, dtype=torch.int32, device=DEV)
    fi = torch.full((I,), 0x7fffffff, dtype=torch.int32, device=DEV)
    out = torch.empty(6 * B, dtype=torch.int64, device=DEV)
    P, st = _lib.ptr, _lib.stream_handle()
    _lib.call("bbgr_ego_slots", B, P(du), P(dp), P(dn), U, I, P(fu), P(fi), P(out), P(out[B:]),
              P(out[3 * B:]), P(out[4 * B:]), P(out[5 * B:]), st)
    iu, cu = out[:B], out[3 * B: 4 * B]
    ue = torch.randn(U, d, generator=g).to(DEV) if U < 5_000_000 else \
        torch.randn(U, d, device=DEV)
    ie = torch.randn(I, d, device=DEV)
    cnt = torch.zeros(3 * B, dtype=torch.int32, device=DEV)
    cnt_u = torch.full((B,), -5, dtype=torch.int32, device=DEV)
    ego = torch.empty(3 * B, d, device=DEV)
    dl = torch.tensor(1.0, device=DEV)
    _lib.call("bbgr_ego_rows", B, d, P(cu), P(out[4 * B:]), P(out[5 * B:]), P(iu), P(out[B:]),
              P(ue), d, P(ie), d, P(dl), 1e-2, P(cnt), P(ego), d, P(ego[B:]), d, 1.0, P(cnt_u), st)
    torch.cuda.synchronize()
    valid = cu >= 0
    # counts: the valid slots pointing at each slot
    want_cnt = torch.bincount(cu[valid], minlength=B)[:B].to(torch.int32)
    assert torch.equal(cnt_u, want_cnt)
    src = torch.randn(B, d, generator=g).to(DEV) * valid[:, None].float()   # invalid: zero rows
    for s in (src, ego[:B]):
        base = torch.randn(U, d, generator=g).to(DEV) if U < 5_000_000 else \
            torch.randn(U, d, device=DEV)
        ref, got = base.clone(), base.clone()
        index_add_rows(ref, iu, s)
        _lib.call("bbgr_rows_add_slots", B, P(cu), P(cnt_u), P(iu), P(s), d, P(got), d, d, U, st)
        torch.cuda.synchronize()
        assert torch.equal(got, ref)
    if B > 1000 and U < 100:   # the case really repeats users (about B / U times each)
        assert int(want_cnt.max()) > 50


@pytest.mark.parametrize("B,U,I", [(1, 3, 2), (8192, 5_000_000, 1_000_000), (4096, 50, 30),
                                   (300, 300, 7)])
def test_ego_slots_kernel_is_the_torch_formulation(B, U, I):
    """bbgr_ego_slots (the drop-in BPR backward's ego-row slots in three
    launches) equals the torch formulation it replaced: clamped ids, the first
    occurrence of each clamped id (bbgr_first_slot semantics, an invalid
    triple's clamped id included), -1 for a triple with any id out of range;
    both scratch tables are left all INT32_MAX."""
    from bbgr import _lib
    g = torch.Generator().manual_seed(B + U + I)
    users = torch.randint(-1, U + 1, (B,), generator=g)
    pos = torch.randint(-1, I + 1, (B,), generator=g)
    neg = torch.randint(-1, I + 1, (B,), generator=g)
    if B > 1000:   # mostly valid, as a sampler's batch
        users, pos, neg = users.clamp(0, U - 1), pos.clamp(0, I - 1), neg.clamp(0, I - 1)
        users[::97], neg[::89] = -1, I
    valid = (users >= 0) & (users < U) & (pos >= 0) & (pos < I) & (neg >= 0) & (neg < I)
    iu = users.clamp(0, U - 1)
    ii = torch.cat([pos, neg]).clamp(0, I - 1)

    def first(ids):
        seen = {}
        return torch.tensor([seen.setdefault(v, b) for b, v in enumerate(ids.tolist())])

    su, si = first(iu), first(ii)
    want_cu = torch.where(valid, su, torch.full_like(su, -1))
    fu = torch.full((U,), 0x7fffffff, dtype=torch.int32, device=DEV)
    fi = torch.full((I,), 0x7fffffff, dtype=torch.int32, device=DEV)
    out = torch.empty(6 * B, dtype=torch.int64, device=DEV)
    du, dp, dn = users.to(DEV), pos.to(DEV), neg.to(DEV)
    for _ in range(2):   # reusable scratch
        out.fill_(-7)
        _lib.call("bbgr_ego_slots", B, _lib.ptr(du), _lib.ptr(dp), _lib.ptr(dn), U, I,
                  _lib.ptr(fu), _lib.ptr(fi), _lib.ptr(out), _lib.ptr(out[B:]), _lib.ptr(out[3 * B:]),
                  _lib.ptr(out[4 * B:]), _lib.ptr(out[5 * B:]), _lib.stream_handle())
        torch.cuda.synchronize()
        o = out.cpu()
        assert torch.equal(o[:B], iu) and torch.equal(o[B:3 * B], ii)
        assert torch.equal(o[3 * B:4 * B], want_cu)
        assert torch.equal(o[4 * B:5 * B], si[:B]) and torch.equal(o[5 * B:], si[B:])
        assert bool((fu == 0x7fffffff).all()) and bool((fi == 0x7fffffff).all())


@pytest.mark.parametrize("ranked", [False, True])
def test_graph_rows_kernel(ranked):
    """bbgr_graph_rows: rank[id] (or the id) inside [0, n), -1 outside."""
    from bbgr import _lib
    n_rows = 1000
    ids = torch.randint(-5, n_rows + 5, (5000,), generator=torch.Generator().manual_seed(3))
    rank = torch.randperm(n_rows, generator=torch.Generator().manual_seed(4))
    ok = (ids >= 0) & (ids < n_rows)
    base = rank[ids.clamp(0, n_rows - 1)] if ranked else ids
    want = torch.where(ok, base, torch.full_like(ids, -1))
    di, dr = ids.to(DEV), rank.to(DEV)
    out = torch.empty_like(di)
    _lib.call("bbgr_graph_rows", ids.numel(), _lib.ptr(di), n_rows,
              _lib.ptr(dr) if ranked else None, _lib.ptr(out), _lib.stream_handle())
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), want)


@pytest.mark.parametrize("d", [16, 64, 256])
def test_rows_add_unique_is_bitwise_the_sorted_scatter(d):
    """bbgr_rows_add_unique (distinct indices, no sort) == bbgr_scatter_add_rows
    bit for bit, signed zeros included (a one-addend segment adds 0 + x), onto
    a zero and a non-zero destination; invalid indices skipped."""
    from bbgr.scatter import RowScatter
    rng = np.random.default_rng(50 + d)
    n_dst = 5000
    idx = rng.permutation(n_dst + 40)[:3000] - 20       # distinct, some out of range
    src = rng.normal(size=(idx.size, d)).astype(np.float32)
    src[:7] = -0.0
    src[7:9] = 0.0
    for base in (np.zeros((n_dst, d), np.float32), rng.normal(size=(n_dst, d)).astype(np.float32)):
        base[:3] = -0.0
        a = RowScatter()(t(base), t(idx, torch.int64), t(src))
        b = RowScatter()(t(base), t(idx, torch.int64), t(src), unique=True)
        np.testing.assert_array_equal(b.cpu().numpy().view(np.uint32),
                                      a.cpu().numpy().view(np.uint32))


@pytest.mark.parametrize("d,n,n_dst", [(d, 20000, 700) for d in (8, 16, 32, 64, 128, 256)]
                         + [(64, 16384, 700), (16, 16384, 1_000_000), (16, 8192, 5_000_000),
                            (16, 4000, 300), (256, 600, 50), (64, 1, 3)])
def test_scatter_add_rows_matches_index_add(d, n, n_dst):
    """bbgr_scatter_add_rows == numpy add.at (sequential ascending order) bit
    for bit on a zero destination; invalid indices skipped; repeatable; from
    one row to 20000, onto tables of up to 5M rows."""
    from bbgr.scatter import index_add_rows
    rng = np.random.default_rng(d + n)
    idx = rng.integers(-3, n_dst + 3, n)          # duplicates + out-of-range rows
    if n_dst > 100_000:                           # a batch's rows: Zipf-like repeats
        idx = np.minimum(rng.zipf(1.3, n) - 1, n_dst + 2)
    idx[:min(500, n // 2)] = 5                    # one long run
    src = rng.normal(size=(n, d)).astype(np.float32)
    want = np.zeros((n_dst, d), np.float32)
    ok = (idx >= 0) & (idx < n_dst)
    np.add.at(want, idx[ok], src[ok])
    got = index_add_rows(torch.zeros(n_dst, d, device=DEV), t(idx, torch.int64), t(src))
    np.testing.assert_array_equal(got.cpu().numpy(), want)
    base = rng.normal(size=(n_dst, d)).astype(np.float32)
    got2 = index_add_rows(t(base), t(idx, torch.int64), t(src)).cpu().numpy()
    np.testing.assert_allclose(got2, base.astype(np.float64) + want, rtol=1e-5, atol=1e-4)
    got3 = index_add_rows(t(base), t(idx, torch.int64), t(src)).cpu().numpy()
    np.testing.assert_array_equal(got2, got3)
    empty = index_add_rows(t(base), torch.empty(0, dtype=torch.int64, device=DEV), t(src))
    np.testing.assert_array_equal(empty.cpu().numpy(), base)


@pytest.mark.parametrize("d,n,n_dst", [(64, 16384, 1_000_000), (16, 3000, 200), (256, 5, 3)])
def test_scatter_plan_applies_like_the_concatenated_scatter(d, n, n_dst):
    """bbgr_scatter_plan + bbgr_scatter_apply: one sort applied to two tables
    gives bbgr_scatter_add_rows' bits each time, and with a second source it
    equals the scatter of [src; src2] over [idx; idx] bit for bit (the drop-in
    backward's item gradient: BPR rows, then ego rows, one sum per item)."""
    import ctypes
    from bbgr import _lib
    from bbgr.scatter import index_add_rows
    rng = np.random.default_rng(n + d)
    idx = np.minimum(rng.zipf(1.2, n) - 1, n_dst + 1)   # repeats + out-of-range rows
    idx[: n // 3] = rng.integers(-2, n_dst + 2, n // 3)
    src = rng.normal(size=(n, d)).astype(np.float32)
    src2 = rng.normal(size=(n, d)).astype(np.float32)
    src2[::3] = 0.0
    di, ds, ds2 = t(idx, torch.int64), t(src), t(src2)
    need = ctypes.c_size_t(0)
    _lib.call("bbgr_scatter_plan", n, _lib.ptr(di), n_dst, None, ctypes.byref(need),
              _lib.stream_handle())
    plan = torch.empty(max(need.value, 1), dtype=torch.uint8, device=DEV)
    _lib.call("bbgr_scatter_plan", n, _lib.ptr(di), n_dst, _lib.ptr(plan), ctypes.byref(need),
              _lib.stream_handle())
    base = rng.normal(size=(n_dst, d)).astype(np.float32)
    for s2 in (None, ds2):
        want = index_add_rows(t(base), di if s2 is None else torch.cat([di, di]),
                              ds if s2 is None else torch.cat([ds, ds2]))
        for _ in range(2):   # the plan is reusable
            got = t(base)
            _lib.call("bbgr_scatter_apply", n, n_dst, _lib.ptr(plan), _lib.ptr(ds), d,
                      None if s2 is None else _lib.ptr(s2), d, _lib.ptr(got), d, d,
                      _lib.stream_handle())
            torch.cuda.synchronize()
            np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32),
                                          want.cpu().numpy().view(np.uint32))


def test_training_step_is_bitwise_reproducible():
    """With the deterministic BPR scatter every reduction of the fused step has
    a fixed order: two trainers from the same state agree bit for bit."""
    from bbgr.synthetic import CONFIGS, config_edges
    from bbgr.trainer import FusedTrainer
    c = CONFIGS["C2"]
    U, I = c["num_users"], c["num_items"]
    g = BipartiteGraph(config_edges("C2"), U, I, DEV)
    kw = dict(cred=synthetic_credibility(U, 2), emb_dim=64, num_layers=3, batch_size=4096,
              seed=9, frontier=True)
    a, b = FusedTrainer(g, "v2_pop", **kw), FusedTrainer(g, "v2_pop", **kw)
    for _ in range(3):
        assert float(a.step()) == float(b.step())
    for x, y in ((a.user_w, b.user_w), (a.item_w, b.item_w), (a.m_u, b.m_u), (a.v_i, b.v_i)):
        assert torch.equal(x, y)


def test_mask_to_list_rows_gather_and_compact_epilogue():
    """The sparse-exchange primitives: mask -> ascending row list (exact),
    row gather (exact copy, zero rows for -1), and the compact epilogue
    (row j of t -> output row list[j]) == the dense epilogue on those rows."""
    import ctypes
    from bbgr._lib import call, ld, ptr, stream_handle
    from bbgr.propagate import epilogue
    rng = np.random.default_rng(11)
    n, d = 5000, 64
    for frac in (0.0, 0.03, 1.0):
        m = (rng.random(n) < frac).astype(np.uint8) * rng.integers(1, 4, n).astype(np.uint8)
        mask = t(m, torch.uint8)
        out = torch.full((n,), -7, dtype=torch.int64, device=DEV)
        cnt = torch.zeros(1, dtype=torch.int64, device=DEV)
        need = ctypes.c_size_t(0)
        call("bbgr_mask_to_list", n, ptr(mask), ptr(out), ptr(cnt), None, ctypes.byref(need),
             stream_handle())
        ws = torch.empty(max(need.value, 1), dtype=torch.uint8, device=DEV)
        call("bbgr_mask_to_list", n, ptr(mask), ptr(out), ptr(cnt), ptr(ws),
             ctypes.byref(need), stream_handle())
        want = np.flatnonzero(m)
        assert int(cnt.item()) == want.size
        np.testing.assert_array_equal(out[: want.size].cpu().numpy(), want)
        # the list split at range boundaries (the sparse exchange's offsets);
        # entries past *count (-7 here) must not be read
        bounds = np.array([0, 1, 17, 2500, want[want.size // 2] if want.size else 9,
                           n - 1, n], np.int64)
        offs = torch.full((bounds.size,), -1, dtype=torch.int64, device=DEV)
        call("bbgr_list_offsets", bounds.size, ptr(t(bounds, torch.int64)), ptr(out), ptr(cnt),
             ptr(offs), stream_handle())
        np.testing.assert_array_equal(offs.cpu().numpy(),
                                      np.searchsorted(want, bounds, side="left"))
        pos = torch.full((n,), -3, dtype=torch.int32, device=DEV)
        call("bbgr_list_positions", n, ptr(out), ptr(cnt), ptr(pos), stream_handle())
        ref = np.full(n, -3, np.int32)
        ref[want] = np.arange(want.size)
        np.testing.assert_array_equal(pos.cpu().numpy(), ref)
    src = t(rng.standard_normal((n, 68)).astype(np.float32))[:, :d]   # ld 68
    idx = t(np.concatenate([rng.integers(0, n, 300), [-1, 0, n - 1]]), torch.int64)
    dst = torch.full((idx.numel(), d), 5.0, device=DEV)
    call("bbgr_rows_gather", idx.numel(), ptr(idx), ptr(src), ld(src), ptr(dst), ld(dst), d,
         stream_handle())
    ref = src.cpu().numpy()[idx.cpu().numpy().clip(0)]
    ref[idx.cpu().numpy() < 0] = 0.0
    np.testing.assert_array_equal(dst.cpu().numpy(), ref)
    # compact epilogue vs dense epilogue restricted to the listed rows
    rows = t(np.sort(rng.choice(n, 400, replace=False)), torch.int64)
    T_full = t(rng.standard_normal((n, d)).astype(np.float32))
    add = t(rng.standard_normal((n, d)).astype(np.float32))
    acc_in = t(rng.standard_normal((n, d)).astype(np.float32))
    ys = t(rng.random(n).astype(np.float32))
    cs = t(rng.random(n).astype(np.float32))
    kw = dict(y_scale=ys, add=add, add_scale_s=0.25, acc_in=acc_in, acc_scale=cs, gamma=0.5)
    y1, a1 = torch.zeros(n, d, device=DEV), torch.zeros(n, d, device=DEV)
    y2, a2 = torch.zeros(n, d, device=DEV), torch.zeros(n, d, device=DEV)
    epilogue(T_full, y=y1, acc_out=a1, **kw)
    comp = T_full[rows].contiguous()
    epilogue(comp, y=y2, acc_out=a2, row_list=rows, n_rows=n, **kw)
    r = rows.cpu().numpy()
    np.testing.assert_array_equal(y2.cpu().numpy()[r], y1.cpu().numpy()[r])
    np.testing.assert_array_equal(a2.cpu().numpy()[r], a1.cpu().numpy()[r])
    other = np.setdiff1d(np.arange(n), r)
    assert not y2.cpu().numpy()[other].any() and not a2.cpu().numpy()[other].any()



@pytest.mark.parametrize("d", [64, 128, 256])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_spmm_pair_rows_match_single_row_path(d, mode, monkeypatch):
    """Two short rows per 16-lane group (low-degree tables) == one row per group,
    bitwise: empty rows, rows spanning several 16-edge batches, chunked long
    rows, src masks, row masks, row lists, row ranges, fused Adam."""
    from bbgr.optim import AdamRows
    from bbgr.propagate import Product, spmm
    rng = np.random.default_rng(200 + d + mode)
    Rn, Cn = 3001, 700
    deg = rng.geometric(0.12, Rn) - 1
    deg[rng.choice(Rn, 6, replace=False)] = [40, 300, 700, 17, 16, 33]
    rows = np.repeat(np.arange(Rn), deg).astype(np.int32)
    cols = rng.integers(0, Cn, rows.size).astype(np.int32)
    vals = rng.uniform(0.1, 1.0, rows.size).astype(np.float32)
    cs = rng.uniform(0.5, 2.0, Cn).astype(np.float32)
    c = Csr(rows, cols, Rn, Cn, DEV, edge_values=t(vals) if mode == 1 else None,
            long_threshold=64, chunk_edges=128)
    prod = Product(c, c.values if mode == 1 else None, t(cs) if mode == 2 else None, None, {})
    x = t(rng.uniform(-1, 1, (Cn, d)).astype(np.float32))
    add = t(rng.normal(size=(Rn, d)).astype(np.float32))
    src_mask = t((rng.random(Cn) < 0.3).astype(np.uint8), torch.uint8)
    row_mask = t((rng.random(Rn) < 0.4).astype(np.uint8), torch.uint8)
    row_list = torch.nonzero(row_mask).flatten()
    p0 = t(rng.normal(size=(Rn, d)).astype(np.float32))

    def run(pair, **kw):
        monkeypatch.setenv("BBGR_SPMM_PAIR", str(pair))
        y = torch.full((Rn, d), 7.0, device=DEV)
        acc = torch.full((Rn, d), 7.0, device=DEV)
        spmm(prod, x, True, y=y, y_scale_s=0.5, add=add, add_scale_s=2.0, acc_out=acc,
             gamma=0.25, **kw)
        torch.cuda.synchronize()
        return y.cpu().numpy(), acc.cpu().numpy()

    cases = [{}, {"src_mask": src_mask}, {"row_mask": row_mask},
             {"row_mask": row_mask, "row_list": row_list}]
    cases += [{"rng": rg} for rg in c.row_ranges(3)]
    for kw in cases:
        a, b = run(0, **kw), run(1, **kw)
        np.testing.assert_array_equal(b[0], a[0], err_msg=f"y {list(kw)}")
        np.testing.assert_array_equal(b[1], a[1], err_msg=f"acc {list(kw)}")
    outs = []
    for pair in (0, 1):   # fused Adam epilogue
        monkeypatch.setenv("BBGR_SPMM_PAIR", str(pair))
        p, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
        spmm(prod, x, True, add=add, add_scale_s=2.0, adam=AdamRows(p, m, v, 1, 1e-3))
        torch.cuda.synchronize()
        outs.append((p.cpu().numpy(), m.cpu().numpy(), v.cpu().numpy()))
    for a, b in zip(*outs):
        np.testing.assert_array_equal(b, a)


@pytest.mark.parametrize("d", [64, 128])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_src_masked_launch_is_bitwise_the_dense_product(d, mode, monkeypatch):
    """A src-masked launch (dead edges skipped) is bitwise the unmasked launch
    over the source table zeroed off the mask, for live fractions 0 .. 1, one-
    and two-row kernels, every weight mode, chunked long rows and row ranges.
    (The slot-bitmap path's live-edge compaction is pinned against the mask by
    test_row_list_with_device_length / the single-chunk boundary test.)"""
    from bbgr.propagate import Product, spmm
    rng = np.random.default_rng(300 + d + mode)
    Rn, Cn = 2500, 900
    deg = rng.geometric(0.1, Rn) - 1
    deg[rng.choice(Rn, 5, replace=False)] = [16, 17, 31, 200, 900]
    rows = np.repeat(np.arange(Rn), deg).astype(np.int32)
    cols = rng.integers(0, Cn, rows.size).astype(np.int32)
    vals = rng.uniform(0.1, 1.0, rows.size).astype(np.float32)
    cs = rng.uniform(0.5, 2.0, Cn).astype(np.float32)
    c = Csr(rows, cols, Rn, Cn, DEV, edge_values=t(vals) if mode == 1 else None,
            long_threshold=64, chunk_edges=128)
    prod = Product(c, c.values if mode == 1 else None, t(cs) if mode == 2 else None, None, {})
    x = rng.uniform(-1, 1, (Cn, d)).astype(np.float32)
    for frac in (0.0, 0.05, 0.41, 0.9, 1.0):
        m = (rng.random(Cn) < frac).astype(np.uint8)
        xm = t(x * m[:, None])
        for pair in (0, 1):
            monkeypatch.setenv("BBGR_SPMM_PAIR", str(pair))
            for rg in [None] + list(c.row_ranges(2)):
                kw = {} if rg is None else {"rng": rg}
                ref = torch.full((Rn, d), 7.0, device=DEV)
                got = torch.full((Rn, d), 7.0, device=DEV)
                spmm(prod, xm, True, y=ref, y_scale_s=0.5, **kw)
                spmm(prod, xm, True, y=got, y_scale_s=0.5, src_mask=t(m, torch.uint8), **kw)
                torch.cuda.synchronize()
                np.testing.assert_array_equal(got.cpu().numpy(), ref.cpu().numpy(),
                                              err_msg=f"frac={frac} pair={pair} rng={rg}")


@pytest.mark.parametrize("n", [1, 31, 32, 33, 1000, 1_000_003])
def test_mask_pack(n):
    """bbgr_mask_pack: bit c & 31 of word c >> 5 is mask[c] != 0 (any nonzero
    byte), the bits past n zero, every word of ceil(n / 32) rewritten; the
    unaligned tail and an odd-offset mask included."""
    from bbgr import _lib
    rng = np.random.default_rng(n)
    m = torch.from_numpy((rng.random(n + 1) < 0.3).astype(np.uint8) * rng.integers(1, 255, n + 1)
                         .astype(np.uint8)).to(DEV)
    for off in (0, 1):
        mask = m[off: off + n]
        words = (n + 31) // 32
        bits = torch.full((words + 1,), -1, dtype=torch.int32, device=DEV)
        _lib.call("bbgr_mask_pack", n, _lib.ptr(mask), _lib.ptr(bits), _lib.stream_handle())
        torch.cuda.synchronize()
        mb = np.zeros(words * 32, dtype=np.uint8)
        mb[:n] = (mask.cpu().numpy() != 0)
        want = (mb.reshape(-1, 32).astype(np.uint64) << np.arange(32, dtype=np.uint64)).sum(1)
        want = want.astype(np.uint32)
        got = bits.cpu().numpy().view(np.uint32)
        np.testing.assert_array_equal(got[:words], want)
        assert got[words] == 0xFFFFFFFF   # nothing written past the last word


@pytest.mark.parametrize("d,mode", [(64, 0), (64, 1), (64, 2), (128, 0), (256, 1), (32, 0)])
def test_src_mask_bits_launch_is_bitwise_the_byte_mask_launch(d, mode, monkeypatch):
    """bbgr_spmm_args.src_mask_bits: the per-edge test on the packed mask gives
    the byte mask's launch bit for bit (live fractions 0 .. 1, one- and
    two-row kernels, every weight mode, chunked long rows, row ranges)."""
    from bbgr import _lib
    from bbgr.propagate import Product, spmm
    rng = np.random.default_rng(900 + d + mode)
    Rn, Cn = 2500, 900
    deg = rng.geometric(0.1, Rn) - 1
    deg[rng.choice(Rn, 5, replace=False)] = [16, 17, 31, 200, 900]
    rows = np.repeat(np.arange(Rn), deg).astype(np.int32)
    cols = rng.integers(0, Cn, rows.size).astype(np.int32)
    vals = rng.uniform(0.1, 1.0, rows.size).astype(np.float32)
    cs = rng.uniform(0.5, 2.0, Cn).astype(np.float32)
    c = Csr(rows, cols, Rn, Cn, DEV, edge_values=t(vals) if mode == 1 else None,
            long_threshold=64, chunk_edges=128)
    prod = Product(c, c.values if mode == 1 else None, t(cs) if mode == 2 else None, None, {})
    x = rng.uniform(-1, 1, (Cn, d)).astype(np.float32)
    bits = torch.zeros(Cn // 32 + 1, dtype=torch.int32, device=DEV)
    for frac in (0.0, 0.05, 0.41, 0.9, 1.0):
        m = t((rng.random(Cn) < frac).astype(np.uint8), torch.uint8)
        _lib.call("bbgr_mask_pack", Cn, _lib.ptr(m), _lib.ptr(bits), _lib.stream_handle())
        xm = t(x) * m[:, None].float()
        for pair in (0, 1):
            monkeypatch.setenv("BBGR_SPMM_PAIR", str(pair))
            for rg in [None] + list(c.row_ranges(2)):
                kw = {} if rg is None else {"rng": rg}
                ref = torch.full((Rn, d), 7.0, device=DEV)
                got = torch.full((Rn, d), 7.0, device=DEV)
                spmm(prod, xm, True, y=ref, y_scale_s=0.5, src_mask=m, **kw)
                spmm(prod, xm, True, y=got, y_scale_s=0.5, src_mask=m, src_mask_bits=bits, **kw)
                torch.cuda.synchronize()
                np.testing.assert_array_equal(got.cpu().numpy(), ref.cpu().numpy(),
                                              err_msg=f"frac={frac} pair={pair} rng={rg}")


@pytest.mark.parametrize("d,mode", [(64, 0), (64, 1), (64, 2), (128, 0), (256, 1)])
def test_tagged_indices_launch_is_bitwise_the_src_masked_launch(d, mode, monkeypatch):
    """bbgr_spmm_args.tag_out: a full two-row launch also writes the column
    indices with bit 31 set off tag_mask, and its product is unchanged;
    src_tagged: a masked launch reading liveness from that copy is bitwise the
    src_mask launch (live fractions 0 .. 1, chunked long rows, every weight
    mode). One-row CSRs refuse both."""
    from bbgr.propagate import Product, spmm
    rng = np.random.default_rng(700 + d + mode)
    Rn, Cn = 2500, 900
    deg = rng.geometric(0.1, Rn) - 1
    deg[rng.choice(Rn, 5, replace=False)] = [16, 17, 31, 200, 900]
    rows = np.repeat(np.arange(Rn), deg).astype(np.int32)
    cols = rng.integers(0, Cn, rows.size).astype(np.int32)
    vals = rng.uniform(0.1, 1.0, rows.size).astype(np.float32)
    cs = rng.uniform(0.5, 2.0, Cn).astype(np.float32)
    c = Csr(rows, cols, Rn, Cn, DEV, edge_values=t(vals) if mode == 1 else None,
            long_threshold=64, chunk_edges=128)
    prod = Product(c, c.values if mode == 1 else None, t(cs) if mode == 2 else None, None, {})
    x = rng.uniform(-1, 1, (Cn, d)).astype(np.float32)
    monkeypatch.setenv("BBGR_SPMM_PAIR", "1")
    idx = c.indices[:c.nnz].long()
    for frac in (0.0, 0.05, 0.41, 0.9, 1.0):
        m = t((rng.random(Cn) < frac).astype(np.uint8), torch.uint8)
        xm = t(x) * m[:, None].float()
        tag = torch.full((c.nnz,), 12345, dtype=torch.int32, device=DEV)
        ref = torch.full((Rn, d), 7.0, device=DEV)
        got = torch.full((Rn, d), 7.0, device=DEV)
        spmm(prod, xm, True, y=ref, y_scale_s=0.5)
        spmm(prod, xm, True, y=got, y_scale_s=0.5, tag_out=tag, tag_mask=m)
        assert torch.equal(got, ref), f"writer frac={frac}"
        want = torch.where(m[idx].bool(), idx, idx | (1 << 31)) & 0xFFFFFFFF
        assert torch.equal(tag.long() & 0xFFFFFFFF, want), f"tags frac={frac}"
        ref.fill_(7.0)
        got.fill_(7.0)
        spmm(prod, xm, True, y=ref, y_scale_s=0.5, src_mask=m)
        spmm(prod, xm, True, y=got, y_scale_s=0.5, src_mask=m, tagged=tag)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(got.cpu().numpy(), ref.cpu().numpy(),
                                      err_msg=f"reader frac={frac}")
    monkeypatch.setenv("BBGR_SPMM_PAIR", "0")
    with pytest.raises(_lib.BbgrError, match="two-row CSR"):
        spmm(prod, t(x), True, y=got, src_mask=m, tagged=tag)


@pytest.mark.parametrize("variant", ["gs", "method_a", "jacobi"])
def test_every_layer_vs_oracle(gold, variant):
    """SURVEY §8(d) parity, per layer k and side: the operators' products
    (bbgr_spmm through BipartiteOperator.mm, the torch.sparse.mm of the
    reference's propagate loop) layer by layer against the float64 oracle's
    layer tables, 1e-5 normwise and max-abs."""
    U, I, E, DUP, D, K, B = (int(x) for x in gold["meta"])
    e, cred, u0, i0 = gold["edges"], gold["cred"], gold["u0"], gold["i0"]
    if variant == "jacobi":
        from bbgr.lightgcn_cu import build_cred_weighted_mats
        item_from_user, user_from_item, _ = build_cred_weighted_mats(e, U, I, cred, DEV)
        A, Bm, _ = R.j_mats(e, U, I, cred)
        _, _, us, is_ = R.propagate_j(A, Bm, u0, i0, K)
        u, i = t(u0), t(i0)
        for k in range(1, K + 1):
            u, i = user_from_item.mm(i), item_from_user.mm(u)      # Jacobi: both from layer k-1
            assert_parity(u, us[k], f"J user layer {k}")
            assert_parity(i, is_[k], f"J item layer {k}")
        return
    if variant == "gs":
        from bbgr.lightgcn_cu_pop import build_message_passing_mats
    else:
        from bbgr.lightgcn_cu_pop_long_tail_exposure import build_message_passing_mats
    M_ui, M_iu = build_message_passing_mats(e, U, I, t(cred), DEV)
    A, Bm = R.gs_mats(e, U, I, cred, method_a=(variant == "method_a"))
    _, _, us, is_ = R.propagate_gs(A, Bm, u0, i0, K)
    u = t(u0)
    for k in range(1, K + 1):
        i = M_iu.mm(u)                                             # GS: item first ...
        u = M_ui.mm(i)                                             # ... users from the NEW items
        assert_parity(i, is_[k], f"{variant} item layer {k}")
        assert_parity(u, us[k], f"{variant} user layer {k}")


def test_spmm_row_list_needs_row_mask_on_chunked_plan():
    """a row list without a row mask on a plan with long-row chunks
    used to skip the listed long rows and let the fix-up sum stale partials;
    the call is now rejected (and still accepted on an unchunked plan)."""
    from bbgr.propagate import Product, spmm
    e = synthetic_edges(300, 50, 6000, 3, items="zipf")
    c = Csr(e[1], e[0], 50, 300, DEV, long_threshold=8, chunk_edges=32)
    assert c.n_chunks > 0 and c.n_split > 0
    prod = Product(c, None, None, None, {})
    x = torch.randn(300, 64, device=DEV)
    y = torch.zeros(50, 64, device=DEV)
    lst = torch.tensor([0, 1, 2], dtype=torch.int64, device=DEV)
    with pytest.raises(_lib.BbgrError, match="INVALID"):
        spmm(prod, x, False, y=y, row_list=lst)
    c2 = Csr(e[1], e[0], 50, 300, DEV, long_threshold=1 << 30)
    assert c2.n_chunks == 0
    spmm(Product(c2, None, None, None, {}), x, False, y=y, row_list=lst)
    want = R.csr64(e[1], e[0], np.ones(e.shape[1]), (50, 300)) @ x.double().cpu().numpy()
    assert_parity(y[:3], want[:3], "listed rows")
    assert not y[3:].any()


def test_mark_rows_skips_out_of_range_indices():
    from bbgr._lib import call, ptr, stream_handle
    mask = torch.zeros(10, dtype=torch.uint8, device=DEV)
    idx = torch.tensor([3, -1, 10, 12, 9], dtype=torch.int64, device=DEV)
    guard = torch.zeros(64, dtype=torch.uint8, device=DEV)   # allocated after: canary
    call("bbgr_mark_rows", 5, ptr(idx), 1, ptr(mask), 10, stream_handle())
    torch.cuda.synchronize()
    assert mask.cpu().tolist() == [0, 0, 0, 1, 0, 0, 0, 0, 0, 1]
    assert not guard.any()


def test_mark_list_flags_and_lists_each_row_once():
    """bbgr_mark_list: the rows a call flags first are listed once each (rows
    already flagged, repeats, negatives and out-of-range ids are not), the
    neighbour form lists N(rows) the same way; list order is free."""
    from bbgr._lib import call, ptr, stream_handle
    rng = np.random.default_rng(3)
    n = 1001                                   # not a multiple of 4: the last word
    mask = torch.zeros((n + 3) // 4 * 4, dtype=torch.uint8, device=DEV)[:n]
    mask[7] = 1                                # already flagged: never listed
    lst = torch.full((n,), -9, dtype=torch.int64, device=DEV)
    cnt = torch.zeros(1, dtype=torch.int64, device=DEV)
    ids = np.concatenate([rng.integers(0, n, 3000), [-1, n, n + 5, 7, 7, n - 1]])
    call("bbgr_mark_list", ids.size, ptr(t(ids, torch.int64)), None, None, ptr(mask), n,
         ptr(lst), ptr(cnt), stream_handle())
    want = np.setdiff1d(np.unique(ids[(ids >= 0) & (ids < n)]), [7])
    k = int(cnt.item())
    assert k == want.size
    np.testing.assert_array_equal(np.sort(lst[:k].cpu().numpy()), want)
    m = mask.cpu().numpy()
    assert set(np.flatnonzero(m)) == set(want) | {7}
    # neighbours of some users in a CSR (many shared columns)
    U, I = 300, n
    e = synthetic_edges(U, I, 6000, 5, items="zipf")
    c = Csr(e[0], e[1], U, I, DEV)
    users = rng.choice(U, 64, replace=False)
    mask2 = torch.zeros((I + 3) // 4 * 4, dtype=torch.uint8, device=DEV)[:I]
    cnt.zero_()
    call("bbgr_mark_list", users.size, ptr(t(users, torch.int64)), ptr(c.indptr),
         ptr(c.indices), ptr(mask2), I, ptr(lst), ptr(cnt), stream_handle())
    ip, ix = c.indptr.cpu().numpy(), c.indices[: c.nnz].cpu().numpy()
    want = np.unique(np.concatenate([ix[ip[u]:ip[u + 1]] for u in users]))
    k = int(cnt.item())
    np.testing.assert_array_equal(np.sort(lst[:k].cpu().numpy()), want)
    np.testing.assert_array_equal(np.flatnonzero(mask2.cpu().numpy()), want)


@pytest.mark.parametrize("bits", [False, True])
def test_row_list_with_device_length(bits):
    """A row list whose length is in device memory (bbgr_spmm_args.row_count,
    capacity = numel): entries past the count are never read, the listed rows
    are bitwise the mask launch's, other rows untouched; with a slot bitmap
    (spmm_bits_kernel) single- and multi-chunk hub rows too."""
    from bbgr._lib import call, ptr, stream_handle
    from bbgr.propagate import Product, spmm
    rng = np.random.default_rng(5)
    U, I, d = 6000, 400, 64
    e = synthetic_edges(U, I, 150000, 6, items="zipf")   # item rows up to ~5k edges
    g = BipartiteGraph(e, U, I, DEV, vertex_order="degree")
    ic = g.item_csr
    prod = Product(ic, None, None, None, {})
    x = torch.zeros(U, d, device=DEV)
    users = rng.choice(U, 200, replace=False)
    x[t(users, torch.int64).long()] = t(rng.standard_normal((200, d)).astype(np.float32))
    su = torch.zeros(U, dtype=torch.uint8, device=DEV)
    su[t(users, torch.int64).long()] = 1
    ri = np.sort(rng.choice(I, 150, replace=False))
    rm = torch.zeros(I, dtype=torch.uint8, device=DEV)
    rm[t(ri, torch.int64).long()] = 1
    kw = dict(src_mask=su, row_mask=rm)
    if bits:
        slots = g.user_item_slots()
        sb = torch.zeros(ic.nnz // 32 + 4, dtype=torch.int32, device=DEV)
        call("bbgr_mark_slots", users.size, ptr(t(users, torch.int64)), ptr(g.user_csr.indptr),
             ptr(slots), ptr(sb), 1, stream_handle())
        kw["src_bits"] = sb
    ref = torch.full((I, d), 3.0, device=DEV)
    spmm(prod, x, False, y=ref, src_mask=su, row_mask=rm)          # mask launch, no bitmap
    lst = torch.full((I,), -5, dtype=torch.int64, device=DEV)      # junk past the count
    lst[: ri.size] = t(rng.permutation(ri), torch.int64).long()
    cnt = torch.tensor([ri.size], dtype=torch.int64, device=DEV)
    y = torch.full((I, d), 3.0, device=DEV)
    spmm(prod, x, False, y=y, row_list=lst, row_count=cnt, **kw)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
    assert ic.n_chunks > 0 and int((ic.degrees() > ic.chunk_edges).sum()) > 0   # both hub kinds


def test_slot_bitmap_single_chunk_boundary_rows_bitwise():
    """spmm_bits_kernel sums single-chunk hub rows (long_threshold < deg <=
    chunk_edges) in one lane group (chunk_row_serial) and longer ones in chunk
    workgroups: rows at both edges of that rule (deg = long_threshold,
    long_threshold + 1, chunk_edges, chunk_edges + 1, 2 * chunk_edges + 1)
    must be bitwise the mask-only launch."""
    from bbgr._lib import call, ptr, stream_handle
    from bbgr.propagate import Product, spmm
    rng = np.random.default_rng(11)
    U, d = 9000, 64
    degs = [64, 65, 2048, 2049, 4097, 40, 3]   # small-graph plan: thr 64, chunk 2048
    rows = np.concatenate([np.full(k, r) for r, k in enumerate(degs)])
    cols = np.concatenate([rng.choice(U, k, replace=False) for k in degs])
    I = len(degs)
    e = np.stack([cols, rows]).astype(np.int32)   # [users; items]
    g = BipartiteGraph(e, U, I, DEV, vertex_order="degree")
    ic = g.item_csr
    assert ic.long_threshold == 64 and ic.chunk_edges == 2048
    prod = Product(ic, None, None, None, {})
    x = torch.zeros(U, d, device=DEV)
    users = rng.choice(U, 3000, replace=False)
    x[t(users, torch.int64).long()] = t(rng.standard_normal((3000, d)).astype(np.float32))
    su = torch.zeros(U, dtype=torch.uint8, device=DEV)
    su[t(users, torch.int64).long()] = 1
    rm = torch.ones(I, dtype=torch.uint8, device=DEV)
    slots = g.user_item_slots()
    sb = torch.zeros(ic.nnz // 32 + 4, dtype=torch.int32, device=DEV)
    call("bbgr_mark_slots", users.size, ptr(t(users, torch.int64)), ptr(g.user_csr.indptr),
         ptr(slots), ptr(sb), 1, stream_handle())
    ref = torch.full((I, d), 3.0, device=DEV)
    spmm(prod, x, False, y=ref, src_mask=su, row_mask=rm)
    lst = torch.arange(I, dtype=torch.int64, device=DEV)
    cnt = torch.tensor([I], dtype=torch.int64, device=DEV)
    y = torch.full((I, d), 3.0, device=DEV)
    spmm(prod, x, False, y=y, row_list=lst, row_count=cnt, src_mask=su, row_mask=rm,
         src_bits=sb)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
    assert sorted(ic.degrees().cpu().tolist(), reverse=True) == sorted(degs, reverse=True)


@pytest.mark.parametrize("n_live", [12, 60, 400])
@pytest.mark.parametrize("weighted", [False, True])
def test_slot_bitmap_sparse_live_rows_bitwise(n_live, weighted):
    """chunk_row_serial's fast path: with few live source rows most of a
    single-chunk row's 16 ranges hold at most one live edge (their terms are
    gathered together and added in range order); with more, some range holds
    two and the row takes the per-range path. Both bitwise the mask-only
    launch, unweighted and with per-edge values (C4's live density is ~1 edge
    in 600)."""
    from bbgr._lib import call, ptr, stream_handle
    from bbgr.propagate import Product, spmm
    rng = np.random.default_rng(n_live)
    U, d = 9000, 64
    degs = [300, 700, 1200, 2048, 2049, 65, 64, 5]
    rows = np.concatenate([np.full(k, r) for r, k in enumerate(degs)])
    cols = np.concatenate([rng.choice(U, k, replace=False) for k in degs])
    I = len(degs)
    e = np.stack([cols, rows]).astype(np.int32)
    g = BipartiteGraph(e, U, I, DEV, vertex_order="degree")
    ic = g.item_csr
    vals = t(rng.uniform(-1.5, 1.5, ic.nnz).astype(np.float32)) if weighted else None
    prod = Product(ic, vals, None, None, {})
    x = torch.zeros(U, d, device=DEV)
    users = rng.choice(U, n_live, replace=False)
    x[t(users, torch.int64).long()] = t(rng.standard_normal((n_live, d)).astype(np.float32))
    su = torch.zeros(U, dtype=torch.uint8, device=DEV)
    su[t(users, torch.int64).long()] = 1
    rm = torch.ones(I, dtype=torch.uint8, device=DEV)
    sb = torch.zeros(ic.nnz // 32 + 4, dtype=torch.int32, device=DEV)
    call("bbgr_mark_slots", users.size, ptr(t(users, torch.int64)), ptr(g.user_csr.indptr),
         ptr(g.user_item_slots()), ptr(sb), 1, stream_handle())
    ref = torch.full((I, d), 3.0, device=DEV)
    spmm(prod, x, False, y=ref, src_mask=su, row_mask=rm)
    y = torch.full((I, d), 3.0, device=DEV)
    spmm(prod, x, False, y=y, row_list=torch.arange(I, dtype=torch.int64, device=DEV),
         row_count=torch.tensor([I], dtype=torch.int64, device=DEV), src_mask=su, row_mask=rm,
         src_bits=sb)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
    assert bool((ref != 3.0).any())


def test_acc_in_map_reads_acc_in_through_its_own_map():
    """bbgr_spmm_args.acc_in_map: acc_out row acc_map[r] = gamma * (cs*T +
    acc_in[acc_in_map[r]]) — the drop-in chain's first / last layer."""
    import ctypes
    from bbgr._lib import SpmmArgs, call, ld, ptr, stream_handle
    rng = np.random.default_rng(9)
    R_, C_, d = 300, 200, 64
    e = synthetic_edges(C_, R_, 4000, 7)
    c = Csr(e[1], e[0], R_, C_, DEV)
    x = rng.standard_normal((C_, d)).astype(np.float32)
    acc_in = rng.standard_normal((R_, d)).astype(np.float32)
    pin, pout = rng.permutation(R_).astype(np.int32), rng.permutation(R_).astype(np.int32)
    a = SpmmArgs()
    a.d = d
    xt, ai = t(x), t(acc_in)
    ao = torch.zeros(R_, d, device=DEV)
    a.x, a.ldx = ptr(xt), ld(xt)
    a.acc_in, a.ldacc_in = ptr(ai), ld(ai)
    a.acc_out, a.ldacc_out = ptr(ao), ld(ao)
    a.acc_scale_s, a.gamma, a.y_scale_s, a.add_scale_s, a.col_scale_s = 0.5, 0.25, 1.0, 1.0, 1.0
    mi, mo = t(pin, torch.int32), t(pout, torch.int32)
    a.acc_in_map, a.acc_map = ptr(mi), ptr(mo)
    call("bbgr_spmm", ctypes.byref(c._struct), ctypes.byref(a), stream_handle())
    T_ = R.csr64(e[1], e[0], np.ones(e.shape[1]), (R_, C_)) @ x.astype(np.float64)
    want = np.zeros((R_, d))
    want[pout] = 0.25 * (0.5 * T_ + acc_in[pin].astype(np.float64))
    assert_parity(ao, want, "acc_in_map")
