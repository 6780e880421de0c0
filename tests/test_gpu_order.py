"""GPU: degree-ordered vertex numbering (BipartiteGraph(vertex_order="degree")).

The order itself is integer work and must be exact (numpy's stable argsort of
the negated degrees); the non-temporal source loads it enables must not change
a single bit of the SpMM; a trainer on the reordered graph must be the same
model as on the input order (parity vs the float64 oracle at 1e-5 on input
ids, as in test_gpu_parity.py)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from bbgr.graph import BipartiteGraph, Csr, VertexOrder  # noqa: E402
from bbgr.synthetic import synthetic_credibility, synthetic_edges  # noqa: E402
from oracle import ref_numpy as R  # noqa: E402

DEV = "cuda"
TOL = 1e-5


def t(a, dtype=torch.float32):
    return torch.as_tensor(np.asarray(a)).to(DEV, dtype)


def rel(got, ref):
    got = got.detach().double().cpu().numpy() if isinstance(got, torch.Tensor) else got
    return np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30)


@pytest.mark.parametrize("n", [1, 7, 1000, 300_000, 2_000_000])
def test_degree_count_and_order_match_numpy(n):
    """(n = 2M: 6M ids, the sort / run-length path of bbgr_degree_count_ws)"""
    from bbgr.graph import _degree_count, _relabel
    rng = np.random.default_rng(n)
    ids = rng.zipf(1.3, size=3 * n + 5).astype(np.int64) % n      # many ties, some zeros
    ids = ids.astype(np.int32)
    deg = _degree_count(t(ids, torch.int32), n)
    want = np.bincount(ids, minlength=n)
    np.testing.assert_array_equal(deg.cpu().numpy(), want)
    o = VertexOrder(deg)
    perm = np.argsort(-want, kind="stable")
    np.testing.assert_array_equal(o.perm.cpu().numpy(), perm)
    rank = np.empty(n, np.int64)
    rank[perm] = np.arange(n)
    np.testing.assert_array_equal(o.rank.cpu().numpy(), rank)
    np.testing.assert_array_equal(_relabel(t(ids, torch.int32), o).cpu().numpy(), rank[ids])
    x = t(rng.normal(size=(n, 3)))
    assert torch.equal(o.rows_to_input(o.rows_to_internal(x)), x)
    # ids grouped by value (an edge list ingested one user at a time): one
    # atomic per run of equal ids in a wave, the same exact counts
    grouped = np.sort(ids, kind="stable")
    np.testing.assert_array_equal(_degree_count(t(grouped, torch.int32), n).cpu().numpy(), want)


def test_ordered_graph_csrs_are_the_relabelled_graph():
    U, I = 900, 400
    e = synthetic_edges(U - 3, I - 3, 12000, 4, items="zipf", duplicates=40)
    g = BipartiteGraph(e, U, I, DEV, vertex_order="degree")
    ru = np.argsort(np.argsort(-np.bincount(e[0], minlength=U), kind="stable"), kind="stable")
    ri = np.argsort(np.argsort(-np.bincount(e[1], minlength=I), kind="stable"), kind="stable")
    e2 = np.stack([ru[e[0]], ri[e[1]]]).astype(np.int32)
    indptr, indices = R.edges_to_user_csr(e2, U)
    np.testing.assert_array_equal(g.user_csr.indptr.cpu().numpy(), indptr)
    np.testing.assert_array_equal(g.user_csr.indices[: g.nnz].cpu().numpy(), indices)
    indptr, indices = R.edges_to_user_csr(e2[::-1].copy(), I)
    np.testing.assert_array_equal(g.item_csr.indptr.cpu().numpy(), indptr)
    np.testing.assert_array_equal(g.item_csr.indices[: g.nnz].cpu().numpy(), indices)
    # internal degrees are non-increasing
    assert (np.diff(np.diff(g.user_csr.indptr.cpu().numpy())) <= 0).all()
    assert (np.diff(np.diff(g.item_csr.indptr.cpu().numpy())) <= 0).all()
    # small tables fit the cache budget and stream nothing; with a smaller
    # budget the hot prefix rule applies
    assert g.user_csr.stream_from(64) == 0 and g.item_csr.stream_out_from(64) == 0
    g.user_csr.hot_bytes = g.item_csr.hot_bytes = 1 << 12
    assert g.user_csr.stream_from(64) > 0 and g.item_csr.stream_from(256) > 0
    assert BipartiteGraph(e, U, I, DEV).user_csr.stream_from(64) == 0
    with pytest.raises(ValueError):
        BipartiteGraph(e, U, I, DEV, vertex_order="random")
    with pytest.raises(ValueError):
        BipartiteGraph(e, U - 10, I, DEV, vertex_order="degree")


@pytest.mark.parametrize("d", [64, 128, 256])
@pytest.mark.parametrize("side", ["item_rows", "user_rows"])
def test_stream_from_loads_leave_results_bitwise_equal(d, side):
    """stream_from / stream_out_from only change the cache policy of the
    gathers and stores: every output bit is equal (one-row and two-row kernels,
    split rows, masks, the fused Adam epilogue)."""
    from bbgr.propagate import Product, spmm
    U, I = 3000, 700
    e = synthetic_edges(U, I, 30000, 11, items="zipf")
    rows, cols, nr, nc = (e[1], e[0], I, U) if side == "item_rows" else (e[0], e[1], U, I)
    c = Csr(rows, cols, nr, nc, DEV, long_threshold=64, chunk_edges=128)
    c.hot_bytes = 1 << 12   # a small budget: these tables would otherwise stay cached
    prod = Product(c, None, None, None, {})
    x = torch.randn(nc, d, device=DEV)
    mask = (torch.rand(nc, device=DEV) < 0.3).to(torch.uint8)
    from bbgr.optim import AdamRows
    outs = []
    p0 = torch.randn(nr, d, device=DEV)
    for ordered in (False, True):
        c.cols_by_degree = c.rows_by_degree = ordered
        assert (c.stream_from(d) > 0) == ordered and (c.stream_out_from(d) > 0) == ordered
        y, acc = torch.empty(nr, d, device=DEV), torch.empty(nr, d, device=DEV)
        ym = torch.zeros(nr, d, device=DEV)
        spmm(prod, x, False, y=y, acc_in=x[:nr] if nr <= nc else None, acc_out=acc)
        spmm(prod, x, False, y=ym, src_mask=mask)
        p, m, v = p0.clone(), torch.full_like(p0, 0.01), torch.full_like(p0, 0.02)
        spmm(prod, x, False, adam=AdamRows(p, m, v, 3, 1e-3))    # fused Adam epilogue
        outs.append((y, acc, ym, p, m, v))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("variant", ["v2_pop", "cu_fair", "method_a"])
def test_ordered_trainer_step_vs_oracle(variant):
    """A step of the trainer on the degree-ordered graph, read back by input id
    (batch(), state_dict()), against the float64 oracle on the input graph."""
    from bbgr.trainer import FusedTrainer
    U, I, d, K = 1200, 500, 64, 3
    e = synthetic_edges(U, I, 16000, 21, items="zipf", duplicates=25)
    cred = synthetic_credibility(U, 3)
    rng = np.random.default_rng(4)
    u0 = rng.uniform(-0.3, 0.3, (U, d)).astype(np.float32)
    i0 = rng.uniform(-0.3, 0.3, (I, d)).astype(np.float32)
    lam = 0.05 if variant == "cu_fair" else 0.0
    g = BipartiteGraph(e, U, I, DEV, vertex_order="degree")
    tr = FusedTrainer(g, variant, cred=cred, emb_dim=d, num_layers=K, batch_size=256,
                      u0=u0, i0=i0, lambda_fair=lam, frontier=True)
    deg_u = np.bincount(e[0], minlength=U)
    users_in = np.flatnonzero(deg_u > 0)[::4][:256]
    loss = float(tr.step(t(users_in, torch.int64)))
    uu, pos, neg = (x.cpu().numpy() for x in tr.batch())
    np.testing.assert_array_equal(uu, users_in)
    ind, col = R.edges_to_user_csr(e, U)
    for u, p, n in zip(uu, pos, neg):      # sampler invariants on input ids
        row = col[ind[u]:ind[u + 1]]
        assert p in row and n not in row
    if variant == "cu_fair":
        A, Bm, deg_i = R.j_mats(e, U, I, cred)
        uf, itf, _, _ = R.propagate_j(A, Bm, u0, i0, K)
        pop = deg_i / max(deg_i.max(), 1.0)
    else:
        A, Bm = R.gs_mats(e, U, I, cred, method_a=(variant == "method_a"))
        uf, itf, _, _ = R.propagate_gs(A, Bm, u0, i0, K)
        pop = None
    want, gr = R.bpr_loss(uf, itf, u0, i0, uu, pos, neg, 1e-4, pop, lam)
    assert abs(loss - want) <= TOL * want, (loss, want)
    if variant == "cu_fair":
        gu0, gi0 = R.backward_j(A, Bm, gr["g_uf"], gr["g_if"], K)
    else:
        gu0, gi0 = R.backward_gs(A, Bm, gr["g_uf"], gr["g_if"], K)
    gu0, gi0 = gu0 + gr["g_ue"], gi0 + gr["g_ie"]
    z = np.zeros_like
    pu, _, _ = R.adam_step(u0, gu0, z(gu0), z(gu0), 1)
    pi, _, _ = R.adam_step(i0, gi0, z(gi0), z(gi0), 1)
    sd = tr.state_dict()
    assert rel(sd["user_emb.weight"] - t(u0), pu - u0) <= 1e-4
    assert rel(sd["item_emb.weight"] - t(i0), pi - i0) <= 1e-4
    # the final tables of the updated model, by input id
    pu_f, pi_f = tr.forward()
    u1 = sd["user_emb.weight"].double().cpu().numpy()
    i1 = sd["item_emb.weight"].double().cpu().numpy()
    if variant == "cu_fair":
        ruf, ritf, _, _ = R.propagate_j(A, Bm, u1, i1, K)
    else:
        ruf, ritf, _, _ = R.propagate_gs(A, Bm, u1, i1, K)
    assert rel(pu_f, ruf) <= TOL and rel(pi_f, ritf) <= TOL


def test_default_init_is_the_same_model_in_both_orders():
    """Default (seeded xavier) tables are drawn by input id, so the ordered and
    input-order trainers start from the same model: equal final tables by
    input id up to fp32 summation order, and equal state_dicts bitwise."""
    from bbgr.trainer import FusedTrainer
    U, I, d = 2000, 900, 128
    e = synthetic_edges(U, I, 25000, 8, items="zipf")
    cred = synthetic_credibility(U, 8)
    trs = [FusedTrainer(BipartiteGraph(e, U, I, DEV, vertex_order=o), "v2_pop", cred=cred,
                        emb_dim=d, num_layers=3, batch_size=300, frontier=True) for o in ("input", "degree")]
    sd = [tr.state_dict() for tr in trs]
    for k in sd[0]:
        assert torch.equal(sd[0][k], sd[1][k])
    f = [tr.forward() for tr in trs]
    for a, b in zip(f[0], f[1]):
        assert rel(b, a.double().cpu().numpy()) <= 1e-6


def test_ordered_graph_edge_cases():
    """No edges (identity order, empty CSRs) and isolated rows (numbered last,
    stable by id; their rows survive the state_dict round trip)."""
    from bbgr.trainer import FusedTrainer
    g = BipartiteGraph(np.zeros((2, 0), np.int32), 5, 4, DEV, vertex_order="degree")
    assert g.user_csr.nnz == 0 and g.user_csr.indptr.cpu().tolist() == [0] * 6
    np.testing.assert_array_equal(g.user_order.perm.cpu().numpy(), np.arange(5))
    with pytest.raises(RuntimeError):
        FusedTrainer(g, "v2_pop", emb_dim=64, num_layers=2, batch_size=4)
    U, I = 300, 200
    e = synthetic_edges(U - 40, I - 30, 3000, 2, items="zipf")   # users >= 260, items >= 170 isolated
    g = BipartiteGraph(e, U, I, DEV, vertex_order="degree")
    rank_u = g.user_order.rank.cpu().numpy()
    assert (np.sort(rank_u[U - 40:]) >= U - 40).all() and (np.diff(rank_u[U - 40:]) > 0).all()
    rng = np.random.default_rng(0)
    u0 = rng.normal(size=(U, 64)).astype(np.float32)
    i0 = rng.normal(size=(I, 64)).astype(np.float32)
    tr = FusedTrainer(g, "cu_message", emb_dim=64, num_layers=2, batch_size=64, u0=u0, i0=i0,
                      frontier=True)
    sd = tr.state_dict()
    np.testing.assert_array_equal(sd["user_emb.weight"].cpu().numpy(), u0)
    np.testing.assert_array_equal(sd["item_emb.weight"].cpu().numpy(), i0)
    tr.step()
    sd = tr.state_dict()   # isolated users are never in a batch: untouched by the step
    np.testing.assert_array_equal(sd["user_emb.weight"][U - 40:].cpu().numpy(), u0[U - 40:])


def test_input_order_graph_detects_degree_ordered_ids():
    """A graph handed over already in descending-degree order (ingest.
    degree_relabel) gets the hot-prefix / streaming policy without
    vertex_order="degree"; per side, and only when that side is ordered."""
    from bbgr.ingest import degree_relabel
    U, I = 3000, 700
    e = synthetic_edges(U, I, 30000, 11, items="zipf")
    g = BipartiteGraph(e, U, I, DEV)
    assert not (g.user_csr.cols_by_degree or g.item_csr.cols_by_degree
                or g.user_csr.rows_by_degree or g.item_csr.rows_by_degree)
    e2, _, _ = degree_relabel(e, U, I)
    g2 = BipartiteGraph(e2, U, I, DEV)
    assert g2.user_csr.rows_by_degree and g2.user_csr.cols_by_degree
    assert g2.item_csr.rows_by_degree and g2.item_csr.cols_by_degree
    g2.user_csr.hot_bytes = g2.item_csr.hot_bytes = 1 << 12
    assert g2.user_csr.stream_from(64) > 0 and g2.item_csr.stream_from(64) > 0
    e3 = np.stack([e[0], e2[1]]).astype(np.int32)   # items ordered, users not
    g3 = BipartiteGraph(e3, U, I, DEV)
    assert g3.item_csr.rows_by_degree and g3.user_csr.cols_by_degree
    assert not (g3.user_csr.rows_by_degree or g3.item_csr.cols_by_degree)


def test_dropin_on_degree_relabelled_ids_matches_original():
    """The drop-in model on ingest.degree_relabel'd ids (weights and
    credibility permuted alike) gives the original model's final tables and
    weight gradients, rows mapped back (fp32 rounding: the neighbour order
    inside a row follows the ids)."""
    from bbgr import lightgcn_cu_pop as V2
    from bbgr.ingest import degree_relabel
    U, I, d, K = 3000, 700, 64, 3
    e = synthetic_edges(U, I, 30000, 11, items="zipf")
    cred = torch.as_tensor(synthetic_credibility(U, 3))
    e2, uid, iid = degree_relabel(e, U, I)
    uid_t, iid_t = torch.as_tensor(uid, device=DEV), torch.as_tensor(iid, device=DEV)
    a = V2.LightGCN(U, I, d, K, *V2.build_message_passing_mats(e, U, I, cred, DEV)).to(DEV)
    b = V2.LightGCN(U, I, d, K, *V2.build_message_passing_mats(
        e2, U, I, cred[torch.as_tensor(uid)], DEV)).to(DEV)
    assert b.M_ui.graph.user_csr.cols_by_degree and b.M_ui.graph.user_csr.rows_by_degree
    with torch.no_grad():
        b.user_emb.weight.copy_(a.user_emb.weight[uid_t])
        b.item_emb.weight.copy_(a.item_emb.weight[iid_t])
    g = torch.Generator().manual_seed(2)
    users = torch.randint(0, U, (256,), generator=g).to(DEV)
    pos = torch.randint(0, I, (256,), generator=g).to(DEV)
    neg = torch.randint(0, I, (256,), generator=g).to(DEV)
    ru = torch.argsort(uid_t)   # original id -> new id
    ri = torch.argsort(iid_t)
    def rel(x, y):
        return float((x - y).detach().norm() / y.detach().norm())

    ua, ia = a.get_user_item_emb()
    ub, ib = b.get_user_item_emb()
    assert rel(ub[ru], ua) < 1e-6 and rel(ib[ri], ia) < 1e-6
    a.bpr_loss(users, pos, neg, ua, ia, 1e-4).backward()
    b.bpr_loss(ru[users], ri[pos], ri[neg], ub, ib, 1e-4).backward()
    assert rel(b.user_emb.weight.grad[ru], a.user_emb.weight.grad) < 1e-6
    assert rel(b.item_emb.weight.grad[ri], a.item_emb.weight.grad) < 1e-6


@pytest.mark.parametrize("family", ["v2", "method_a", "cu", "sym"])
def test_dropin_degree_graph_is_bitwise_the_input_order_graph(family, monkeypatch):
    """The drop-in builders number their graph by descending degree
    (operators.DROPIN_VERTEX_ORDER) while every table the caller sees stays in
    input order (first products gather through input-id columns, epilogues
    place rows through maps). Each row keeps its input-order column sequence,
    so the operators' products, the final tables, the per-layer Jacobi op, the
    loss and every weight gradient — through the sparse-rows backward and the
    dense propagate_backward op — are bitwise those of an input-order graph."""
    from bbgr import lightgcn as L
    from bbgr import lightgcn_cu as J
    from bbgr import lightgcn_cu_pop as V2
    from bbgr import lightgcn_cu_pop_long_tail_exposure as MA
    from bbgr import operators, ops
    U, I, d, K, B = 3000, 700, 64, 3, 512
    e = synthetic_edges(U, I, 30000, 11, items="zipf", duplicates=40)
    cred = torch.as_tensor(synthetic_credibility(U, 3))
    g = torch.Generator().manual_seed(5)
    users = torch.randint(0, U, (B,), generator=g).to(DEV)
    pos = torch.randint(0, I, (B,), generator=g).to(DEV)
    neg = torch.randint(0, I, (B,), generator=g).to(DEV)
    gU = torch.zeros(U, d, device=DEV)
    gI = torch.zeros(I, d, device=DEV)
    gU[users] = torch.randn(B, d, generator=g).to(DEV)
    gI[pos] = torch.randn(B, d, generator=g).to(DEV)
    x_u = torch.randn(U, d, generator=g).to(DEV)
    x_i = torch.randn(I, d, generator=g).to(DEV)
    out = {}
    for order in ("input", "degree"):
        monkeypatch.setattr(operators, "DROPIN_VERTEX_ORDER", order)
        torch.manual_seed(0)
        r = []
        if family in ("v2", "method_a"):
            mod = V2 if family == "v2" else MA
            M_ui, M_iu = mod.build_message_passing_mats(e, U, I, cred, DEV)
            m = mod.LightGCN(U, I, d, K, M_ui, M_iu).to(DEV)
            ops_ = (M_iu, M_ui)
            uf, itf = m.propagate()
            loss = m.bpr_loss(users, pos, neg, uf, itf, 1e-4)
        elif family == "cu":
            a, b, deg_i = J.build_cred_weighted_mats(e, U, I, cred, DEV)
            m = J.CredLightGCN(U, I, d, K, a, b).to(DEV)
            ops_ = (a, b)
            r.append(torch.as_tensor(deg_i))
            us, is_ = m.propagate_all_layers()
            r += list(us) + list(is_)
            uf, itf = m.final_embeddings()
            pop = torch.as_tensor(deg_i / deg_i.max(), device=DEV)
            loss = m.bpr_fair_loss(users, pos, neg, uf, itf, pop, 0.05, 1e-4) + \
                sum(t.sum() for t in us[1:]) * 1e-3
        else:
            A = L.build_norm_adj(e, U, I, DEV)
            m = L.LightGCN(U, I, d, K, A).to(DEV)
            ops_ = ()
            r.append(A.to_torch_sparse().to_dense())
            uf, itf = m.get_user_item_emb()
            loss = m.bpr_loss(users, pos, neg, uf, itf, 1e-4)
        graph = getattr(ops_[0], "graph", None) if ops_ else m.norm_adj.graph
        assert (graph.user_order is not None) == (order == "degree")
        for op in ops_:
            r.append(op.mm(x_u if op.shape[1] == U else x_i))
            r.append(op.to_torch_sparse().to_dense())
        loss.backward()
        r += [uf.detach(), itf.detach(), loss.detach()] + [p.grad for p in m.parameters()]
        if family != "sym":   # the dense (registered) backward op, its own masks
            pair = m._operator_pair()
            r += list(ops.propagate_backward(gU, gI, ops.pair_key(pair), K,
                                             "jacobi" if family == "cu" else "gs"))
        out[order] = r
    assert len(out["input"]) == len(out["degree"])
    for k, (a, b) in enumerate(zip(out["input"], out["degree"])):
        assert torch.equal(a.cpu(), b.cpu()), f"{family}: result {k} differs"
