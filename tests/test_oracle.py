"""CPU tests of the oracle (the checker): hand-derived known answers, the two
independent restatements against each other, and algebraic properties.

The reference ships no tests or fixtures and importing it was
refused, so the known answers below are derived by hand from the
reference source lines cited in oracle/ref_numpy.py.
"""
import math

import numpy as np
import pytest
import torch

from oracle import ref_numpy as R
from oracle import ref_torch as T

S2 = 1.0 / math.sqrt(2.0)


def test_kat_gs_operator_and_one_layer():
    # U=2, I=2, edges (0,0),(0,1),(1,1): deg_u=[2,1], deg_i=[1,2]
    e = np.array([[0, 0, 1], [0, 1, 1]], np.int32)
    cred = np.array([1.0, 0.5], np.float32)
    M_ui, M_iu = R.gs_mats(e, 2, 2, cred)
    np.testing.assert_allclose(M_ui.toarray(), [[S2, 0.5], [0.0, S2]], rtol=1e-7)
    np.testing.assert_allclose(M_iu.toarray(), [[S2, 0.0], [0.5, 0.5 * S2]], rtol=1e-7)
    u0, i0 = np.array([[1.0], [2.0]]), np.array([[3.0], [4.0]])
    uf, itf, us, is_ = R.propagate_gs(M_ui, M_iu, u0, i0, 1)
    i1 = np.array([S2, 0.5 + S2])
    u1 = np.array([S2 * S2 + 0.5 * (0.5 + S2), S2 * (0.5 + S2)])
    np.testing.assert_allclose(is_[1].ravel(), i1, rtol=1e-7)
    np.testing.assert_allclose(us[1].ravel(), u1, rtol=1e-7)   # GS: u1 uses the NEW i1
    np.testing.assert_allclose(uf.ravel(), (np.array([1.0, 2.0]) + u1) / 2, rtol=1e-7)
    np.testing.assert_allclose(itf.ravel(), (np.array([3.0, 4.0]) + i1) / 2, rtol=1e-7)


def test_kat_jacobi_uses_old_item_table():
    e = np.array([[0, 0, 1], [0, 1, 1]], np.int32)
    cred = np.array([1.0, 0.5], np.float32)
    M_item_from_user, M_user_from_item, deg_i = R.j_mats(e, 2, 2, cred)
    np.testing.assert_allclose(deg_i, [1.0, 2.0])
    # Eq 3.23: c_u / sqrt(deg_u deg_i); Eq 3.24: 1/sqrt(deg_u deg_i)
    np.testing.assert_allclose(M_item_from_user.toarray(), [[S2, 0.0], [0.5, 0.5 * S2]],
                               rtol=1e-7)
    np.testing.assert_allclose(M_user_from_item.toarray(), [[S2, 0.5], [0.0, S2]], rtol=1e-7)
    u0, i0 = np.array([[1.0], [2.0]]), np.array([[3.0], [4.0]])
    uf, itf, us, is_ = R.propagate_j(M_item_from_user, M_user_from_item, u0, i0, 1)
    np.testing.assert_allclose(us[1].ravel(), [3 * S2 + 2.0, 4 * S2], rtol=1e-7)  # from i0


def test_kat_duplicate_edge_is_summed():
    # (0,0) twice + (1,0): deg_u = [2,1], deg_i = [3] (bincount counts the repeat);
    # coalesce sums -> M_ui[0,0] = 2 * (1/sqrt2 * 1/sqrt3), M_ui[1,0] = 1/sqrt3
    e = np.array([[0, 0, 1], [0, 0, 0]], np.int32)
    want = [[2.0 / math.sqrt(6.0)], [1.0 / math.sqrt(3.0)]]
    M_ui, M_iu = R.gs_mats(e, 2, 1)
    np.testing.assert_allclose(M_ui.toarray(), want, rtol=1e-7)
    Mt_ui, Mt_iu = T.gs_operators(e, 2, 1)
    np.testing.assert_allclose(Mt_ui.to_dense().numpy(), want, rtol=1e-6)


def test_kat_isolated_item_keeps_only_layer0():
    e = np.array([[0], [1]], np.int32)  # U=1, I=3; items 0 and 2 isolated
    M_ui, M_iu = R.gs_mats(e, 1, 3)
    u0, i0 = np.array([[1.0]]), np.array([[5.0], [6.0], [7.0]])
    uf, itf, _, _ = R.propagate_gs(M_ui, M_iu, u0, i0, 3)
    assert itf[0, 0] == pytest.approx(5.0 / 4) and itf[2, 0] == pytest.approx(7.0 / 4)


def test_kat_symmetric_two_nodes():
    e = np.array([[0], [0]], np.int32)  # N=2, A = [[0,1],[1,0]], deg = 1
    A = R.sym_values(e, 1, 1)
    np.testing.assert_allclose(A.toarray(), [[0, 1], [1, 0]])
    xf, _ = R.propagate_sym(A, np.array([[1.0], [2.0]]), 2)
    np.testing.assert_allclose(xf.ravel(), [4 / 3, 5 / 3], rtol=1e-12)
    At = T.sym_operator(e, 1, 1)
    np.testing.assert_allclose(At.to_dense().numpy(), [[0, 1], [1, 0]])


def test_kat_sym_isolated_node_inf_to_zero():
    e = np.array([[0], [0]], np.int32)  # U=2: user 1 isolated -> deg^-1/2 = inf -> 0
    A = R.sym_values(e, 2, 1)
    assert A.shape == (3, 3) and A[1].nnz == 0


def test_kat_method_a_alpha():
    e = np.array([[0, 1, 2], [0, 0, 1]], np.int32)  # deg_i = [2, 1]
    u, i, w_ui, w_iu = R.gs_values(e, 3, 2, None, method_a=True)
    alpha0 = 1.0 / math.log1p(2.0)
    alpha1 = 1.0 / math.log1p(1.0)
    np.testing.assert_allclose(w_ui, [S2 * alpha0, S2 * alpha0, 1.0 * alpha1], rtol=1e-6)


def test_kat_ln2_loss_at_zero_embeddings():
    B, d = 8, 4
    z_u, z_i = np.zeros((3, d)), np.zeros((5, d))
    users = np.arange(B) % 3
    pos, neg = np.arange(B) % 5, (np.arange(B) + 1) % 5
    loss, _ = R.bpr_loss(z_u, z_i, z_u, z_i, users, pos, neg, reg=1e-4)
    assert loss == pytest.approx(math.log(2.0), abs=1e-11)


def _random_case(seed=0, U=60, I=40, E=400, d=8, dup=10):
    from bbgr.synthetic import synthetic_edges
    e = synthetic_edges(U, I, E, seed, items="zipf", duplicates=dup)
    rng = np.random.default_rng(seed)
    cred = rng.uniform(0, 1, U).astype(np.float32)
    u0 = rng.uniform(-1, 1, (U, d)).astype(np.float32)
    i0 = rng.uniform(-1, 1, (I, d)).astype(np.float32)
    return e, cred, u0, i0


def nrel(a, b):
    return np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-300)


@pytest.mark.parametrize("method_a", [False, True])
def test_numpy_vs_torch_gs(method_a):
    e, cred, u0, i0 = _random_case(1)
    M_ui, M_iu = R.gs_mats(e, 60, 40, cred, method_a)
    uf, itf, _, _ = R.propagate_gs(M_ui, M_iu, u0, i0, 3)
    Tui, Tiu = T.gs_operators(e, 60, 40, cred, method_a)
    tuf, titf = T.propagate_gs(Tui, Tiu, torch.tensor(u0), torch.tensor(i0), 3)
    assert nrel(tuf.numpy(), uf) < 1e-6 and nrel(titf.numpy(), itf) < 1e-6


def test_numpy_vs_torch_jacobi_and_sym():
    e, cred, u0, i0 = _random_case(2)
    A, B_, _ = R.j_mats(e, 60, 40, cred)
    uf, itf, _, _ = R.propagate_j(A, B_, u0, i0, 3)
    TA, TB = T.j_operators(e, 60, 40, cred)
    tuf, titf = T.propagate_j(TA, TB, torch.tensor(u0), torch.tensor(i0), 3)
    assert nrel(tuf.numpy(), uf) < 1e-6 and nrel(titf.numpy(), itf) < 1e-6
    S = R.sym_values(e, 60, 40)
    x0 = np.concatenate([u0, i0])
    xf, _ = R.propagate_sym(S, x0, 3)
    txf = T.propagate_sym(T.sym_operator(e, 60, 40), torch.tensor(x0), 3)
    assert nrel(txf.numpy(), xf) < 1e-6


def test_backward_gs_matches_torch_autograd():
    e, cred, u0, i0 = _random_case(3)
    M_ui, M_iu = R.gs_mats(e, 60, 40, cred)
    rng = np.random.default_rng(5)
    gU, gI = rng.normal(size=u0.shape), rng.normal(size=i0.shape)
    gu0, gi0 = R.backward_gs(M_ui, M_iu, gU, gI, 3)
    Tui, Tiu = T.gs_operators(e, 60, 40, cred)
    tu = torch.tensor(u0, dtype=torch.float64, requires_grad=True)
    ti = torch.tensor(i0, dtype=torch.float64, requires_grad=True)
    tuf, titf = T.propagate_gs(Tui.double(), Tiu.double(), tu, ti, 3)
    ((tuf * torch.tensor(gU)).sum() + (titf * torch.tensor(gI)).sum()).backward()
    assert nrel(tu.grad.numpy(), gu0) < 1e-12 and nrel(ti.grad.numpy(), gi0) < 1e-12


def test_backward_jacobi_and_sym_adjoint():
    e, cred, u0, i0 = _random_case(4)
    A, B_, _ = R.j_mats(e, 60, 40, cred)
    rng = np.random.default_rng(6)
    gU, gI = rng.normal(size=u0.shape), rng.normal(size=i0.shape)
    gu0, gi0 = R.backward_j(A, B_, gU, gI, 3)
    uf, itf, _, _ = R.propagate_j(A, B_, u0, i0, 3)
    # propagation is linear: <final, g> == <x0, grad_x0>
    lhs = (uf * gU).sum() + (itf * gI).sum()
    rhs = (u0 * gu0).sum() + (i0 * gi0).sum()
    assert lhs == pytest.approx(rhs, rel=1e-10)
    S = R.sym_values(e, 60, 40)
    x0 = np.concatenate([u0, i0]).astype(np.float64)
    g = rng.normal(size=x0.shape)
    xf, _ = R.propagate_sym(S, x0, 3)
    assert (xf * g).sum() == pytest.approx((x0 * R.backward_sym(S, g, 3)).sum(), rel=1e-10)


def test_bpr_grads_match_torch_autograd():
    rng = np.random.default_rng(7)
    U, I, d, B = 30, 20, 8, 64
    uf, itf, ue, ie = (rng.normal(size=s) for s in ((U, d), (I, d), (U, d), (I, d)))
    users, pos, neg = rng.integers(0, U, B), rng.integers(0, I, B), rng.integers(0, I, B)
    pop = rng.uniform(0, 1, I)
    loss, g = R.bpr_loss(uf, itf, ue, ie, users, pos, neg, 1e-2, pop, 0.3)
    t = [torch.tensor(a, requires_grad=True) for a in (uf, itf, ue, ie)]
    tl = T.bpr(*t, torch.tensor(users), torch.tensor(pos), torch.tensor(neg), 1e-2,
               torch.tensor(pop), 0.3)
    tl.backward()
    assert float(tl.detach()) == pytest.approx(loss, rel=1e-12)
    for k, tt in zip(("g_uf", "g_if", "g_ue", "g_ie"), t):
        assert nrel(tt.grad.numpy(), g[k]) < 1e-10


def test_adam_matches_torch():
    rng = np.random.default_rng(8)
    p0 = rng.normal(size=(16, 4))
    tp = torch.nn.Parameter(torch.tensor(p0))
    opt = torch.optim.Adam([tp], lr=1e-3)
    p, m, v = p0.copy(), np.zeros_like(p0), np.zeros_like(p0)
    for step in range(1, 4):
        g = rng.normal(size=p0.shape)
        tp.grad = torch.tensor(g)
        opt.step()
        p, m, v = R.adam_step(p, g, m, v, step)
    assert nrel(tp.detach().numpy(), p) < 1e-12


@pytest.mark.parametrize("betas", [(0.9, 0.999), (0.8, 0.99), (0.9, 0.9999)])
def test_bias_correction_table_is_exact_past_its_end(betas):
    """The device step state's kernels clamp t to the table end:
    exact because from exact_table_steps() on every step's fp32 constants are
    (1.0f, 1.0f), the value the host computes for any later t."""
    import math
    from bbgr.optim import bias_corrections, exact_table_steps
    b1, b2 = betas
    n = exact_table_steps(b1, b2)
    tab = bias_corrections(n + 64, b1, b2)
    assert np.all(tab[n - 1:] == np.float32(1.0))
    for t in (n, n + 1, 10 * n, 1 << 40):      # the host path's scalars for a later step
        assert np.float32(1.0 - b1 ** t) == tab[n - 1, 0]
        assert np.float32(math.sqrt(1.0 - b2 ** t)) == tab[n - 1, 1]


def test_reference_style_sampler_never_returns_positive():
    e, _, _, _ = _random_case(9, U=50, I=30, E=600, dup=0)
    indptr, indices = R.edges_to_user_csr(e, 50)
    pp = R.pop_prob(e, 30)
    assert pp.sum() == pytest.approx(1.0, abs=1e-9)
    rng = np.random.default_rng(42)
    # the reference loops forever for a user holding every item; skip those
    users = np.flatnonzero(np.diff(indptr) < 30)
    used, pos, neg = R.sample_batch_reference_style(indptr, indices, users, 30, rng, pp)
    for u, p, n in zip(used, pos, neg):
        assert R.user_has_item(indptr, indices, u, p)
        assert not R.user_has_item(indptr, indices, u, n)


def test_edges_to_user_csr_sorted_rows():
    e = np.array([[2, 0, 2, 1, 0], [3, 1, 0, 2, 0]], np.int32)
    indptr, indices = R.edges_to_user_csr(e, 4)
    assert indptr.tolist() == [0, 2, 3, 5, 5]
    assert indices.tolist() == [0, 1, 2, 0, 3]


def test_edges_to_user_csr_equals_the_reference_loop():
    """The oracle's CSR (sorted (user, item) keys) is the array the reference's
    own loop builds (Version-2/lighgcn_cu_pop.py:309-327: mergesort by user,
    then np.sort of each row), written out literally here; with duplicates,
    empty rows and an unsorted input order."""
    rng = np.random.default_rng(7)
    U, I = 60, 25
    e = np.stack([rng.integers(0, U - 5, 900), rng.integers(0, I, 900)]).astype(np.int32)
    e = np.concatenate([e, e[:, :40]], 1)[:, rng.permutation(940)]
    u, it = e[0].astype(np.int64), e[1].astype(np.int64)
    order = np.argsort(u, kind="mergesort")
    u, it = u[order], it[order]
    indptr = np.zeros(U + 1, dtype=np.int64)
    indptr[1:] = np.cumsum(np.bincount(u, minlength=U))
    indices = it.copy()
    for user in range(U):
        a, b = indptr[user], indptr[user + 1]
        if b - a > 1:
            indices[a:b] = np.sort(indices[a:b])
    got_ptr, got_idx = R.edges_to_user_csr(e, U)
    np.testing.assert_array_equal(got_ptr, indptr)
    np.testing.assert_array_equal(got_idx, indices)
    assert got_idx.dtype == np.int64 and got_ptr.dtype == np.int64


def test_metrics_at_k_known_answers():
    import math
    p, r, n = R.metrics_at_k([5, 3, 9, 1], {3}, 2)
    assert (p, r) == (0.5, 1.0) and n == pytest.approx(1 / math.log2(3))
    p, r, n = R.metrics_at_k([5, 3, 9, 1], {7}, 4)
    assert (p, r, n) == (0.0, 0.0, 0.0)
    p, r, n = R.metrics_at_k([3, 5], {3, 5, 8}, 2)
    assert p == 1.0 and r == pytest.approx(2 / 3) and n == pytest.approx(1.0)


def test_evaluate_sampled_given_hand_case():
    uf = np.array([[1.0, 0.0]])
    itf = np.array([[0.9, 0], [0.5, 0], [1.0, 0], [0.1, 0]])
    # cand = [pos=0, 1, 2, 3]; scores .9 .5 1 .1 -> ranked 2,0,1,3: pos at rank 1
    res = R.evaluate_sampled_given([0], [[0, 1, 2, 3]], uf, itf, np.array([0, 1, 2, 3]),
                                   10, 4, np.array([0.5]), [0], [], Ks=(1, 2))
    assert res[1]["recall"] == 0.0 and res[2]["recall"] == 1.0
    assert res[2]["ndcg"] == pytest.approx(1 / np.log2(3))
    assert res[2]["item_coverage"] == 0.5 and res[2]["high_cred_recall"] == 1.0


def test_eval_reference_style_invariants():
    """The full reference loop restatement (Version-2:536-650): candidate
    invariants, group sizes, and agreement with evaluate_sampled_given."""
    from bbgr.synthetic import synthetic_edges
    U, I, d = 300, 400, 16
    e = synthetic_edges(U, I, 4000, 2)
    rng = np.random.default_rng(0)
    m = rng.random(e.shape[1]) < 0.2
    tr, te = e[:, ~m], e[:, m]
    trp, tri = R.edges_to_user_csr(tr, U)
    tep, tei = R.edges_to_user_csr(te, U)
    uf = rng.normal(size=(U, d)).astype(np.float32)
    itf = rng.normal(size=(I, d)).astype(np.float32)
    pop = np.bincount(tr[1], minlength=I)
    cred = rng.random(U)
    res, cands = R.evaluate_sampled_reference_style(trp, tri, tep, tei, uf, itf, I, pop,
                                                    tr.shape[1], cred)
    users = np.where(np.diff(tep) > 0)[0]
    assert len(cands) == users.size and all(len(c) == 100 for c in cands)
    for u, c in zip(users, cands):
        assert R.user_has_item(tep, tei, u, c[0])
        assert not any(R.user_has_item(tep, tei, u, j) or R.user_has_item(trp, tri, u, j)
                       for j in c[1:])
    k = max(int(round(users.size * 0.2)), 1)
    assert res[10]["high_users"] == res[10]["low_users"] == k
    hi, lo = R.make_cred_groups(users, cred, 0.2)
    assert cred[hi].min() >= cred[lo].max()
    again = R.evaluate_sampled_given(users, np.asarray(cands), uf, itf, pop, tr.shape[1], I,
                                     cred, hi, lo)
    assert again[20]["ndcg"] == res[20]["ndcg"]
    assert 0.0 <= res[10]["recall"] <= res[20]["recall"] <= 1.0


def test_full_ranking_c_oracle():
    """oracle/csrc/eval_full.c: the fma-chain score agrees with float64 to fp32
    rounding; its top-k equals the reference-style numpy ranking
    (Version-2:690-706) except where two scores are within fp32 noise; train
    items sink to -1e9; users with < k untrained items get -1e9 entries."""
    from oracle import native as N
    rng = np.random.default_rng(5)
    U, I, d, k = 60, 300, 64, 20
    uf = rng.normal(size=(U, d)).astype(np.float32)
    itf = rng.normal(size=(I, d)).astype(np.float32)
    for _ in range(20):
        a, b = rng.normal(size=d).astype(np.float32), rng.normal(size=d).astype(np.float32)
        exact = float(np.dot(a.astype(np.float64), b.astype(np.float64)))
        assert abs(N.score_chain(a, b) - exact) <= 1e-6 * np.abs(a * b).sum()
    tr = []
    for u in range(U):
        n = 295 if u == 0 else rng.integers(0, 15)          # user 0: only 5 untrained items
        tr.append(np.sort(rng.choice(I, n, replace=False)))
    ptr = np.concatenate([[0], np.cumsum([len(t) for t in tr])]).astype(np.int32)
    idx = np.concatenate(tr).astype(np.int32)
    users = np.arange(U)
    items, scores = N.full_topk(users, ptr, idx, uf, itf, k)
    ref = R.full_ranking_reference_style(users, ptr, idx, uf, itf, k)
    same = (items == ref).all(axis=1)
    assert same.mean() >= 0.95
    for b in np.where(~same)[0]:                            # only near-ties may differ
        s_ref = np.sort((uf[b] @ itf.T.astype(np.float64))[ref[b]])[::-1]
        assert np.allclose(np.sort(scores[b])[::-1][:5], s_ref[:5], rtol=1e-5, atol=1e-5)
    assert (scores[0, 5:] == np.float32(-1e9)).all() and not np.isin(items[0, :5], tr[0]).any()
    for b in range(1, U):
        assert not np.isin(items[b], tr[b]).any()
        assert (np.diff(scores[b]) <= 0).all()


def test_cred_gnn_oracle_known_answers():
    """main.py:677-691 restated: EWA clamps, per-dst normalisation sums to 1
    over each destination with positive weight, aggregation by hand; the numpy
    and torch restatements agree."""
    import torch
    from oracle import ref_torch as T
    ea = np.array([[1.5, 0.2, 0, 0, 0], [0.0, -0.5, 0, 0, 0], [0.5, 0.25, 0, 0, 0],
                   [-1.0, 2.0, 0, 0, 0]], np.float32)
    w = R.ewa_raw(ea)
    np.testing.assert_allclose(w, [1.2, 0.0, 0.75, 2.0], rtol=1e-7)
    ei = np.array([[0, 1, 2, 2], [0, 0, 0, 1]])
    wt = R.normalize_per_dst(w, ei[1], 3)
    np.testing.assert_allclose(wt, [1.2 / 1.95, 0.0, 0.75 / 1.95, 1.0], rtol=1e-6)
    x = np.array([[1.0, 0.0], [0.0, 1.0], [2.0, 2.0]])
    agg = R.aggregate(x, ei, wt, 3)
    np.testing.assert_allclose(agg[0], [1.2 / 1.95 + 1.5 / 1.95, 1.5 / 1.95], rtol=1e-6)
    np.testing.assert_allclose(agg[1], [2.0, 2.0]) and np.testing.assert_allclose(agg[2], 0.0)
    m = T.CredModelRef(3, 3, 4)
    tw = m.normalize_per_dst(m.ewa_raw(torch.tensor(ea)), torch.tensor(ei[1]), 3)
    np.testing.assert_allclose(tw.numpy(), wt, rtol=1e-6)
    ta = m.aggregate(torch.tensor(x, dtype=torch.float32), torch.tensor(ei), tw, 3)
    np.testing.assert_allclose(ta.numpy(), agg, rtol=1e-6)


def test_rows_product_equals_full_product_rows():
    """The sampled-row evaluator of the full-size parity tests equals the rows
    of the whole float64 product (duplicates, empty rows, unsorted selection)."""
    rng = np.random.default_rng(5)
    rows = rng.integers(0, 60, 2000)
    cols = rng.integers(0, 40, 2000)
    w = rng.random(2000).astype(np.float32)
    x = rng.normal(size=(40, 16))
    sel = np.array([59, 3, 0, 17, 48, 12])
    rows[rows == 12] = 13                      # row 12 has no edges
    m = np.isin(rows, sel)
    got = R.rows_product(sel, rows[m], cols[m], w[m], x[cols[m]])
    want = (R.csr64(rows, cols, w, (60, 40)) @ x)[sel]
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12)
    assert not got[sel == 12].any()


def test_edge_weights_match_operator_builders():
    """edge_weights on an edge subset equals the full builders' values."""
    e = np.array([[0, 0, 1, 2, 2, 2], [0, 1, 1, 0, 1, 3]], np.int32)
    U, I = 4, 5
    cred = np.array([0.5, 1.0, 0.25, 0.8], np.float32)
    deg_u, deg_i = R.degrees(e, U, I)
    for kind, full in (("gs", R.gs_values(e, U, I, cred)),
                       ("method_a", R.gs_values(e, U, I, cred, method_a=True))):
        a, b = R.edge_weights(kind, e[0], e[1], deg_u, deg_i, cred)
        np.testing.assert_array_equal(a, full[2])
        np.testing.assert_array_equal(b, full[3])
    u, i, w_ui, w_iu, _ = R.j_values(e, U, I, cred)
    a, b = R.edge_weights("j", e[0], e[1], deg_u, deg_i, cred)
    np.testing.assert_array_equal(a, w_iu)
    np.testing.assert_array_equal(b, w_ui)
    S = R.sym_values(e, U, I)
    a, _ = R.edge_weights("sym", e[0], e[1], deg_u, deg_i)
    np.testing.assert_allclose(a, np.asarray(S[e[0], e[1] + U]).ravel(), rtol=1e-7)


@pytest.mark.parametrize("kind,order", [("gs", "gs"), ("method_a", "gs"), ("j", "jacobi")])
def test_chain64_matches_scipy_restatement(kind, order):
    """oracle/chain64 (the C float64 chain the full-size GPU parity tests use)
    equals the scipy restatement (propagate_* / backward_*) on a graph with
    duplicate edges and a hub item: every layer, finals and both gradients."""
    from bbgr.synthetic import synthetic_credibility, synthetic_edges
    from oracle.chain64 import Chain64
    U, I, K = 300, 200, 3
    e = synthetic_edges(U, I, 4000, seed=3, items="zipf", duplicates=30)
    cred = synthetic_credibility(U, 3)
    rng = np.random.default_rng(0)
    u0, i0 = rng.standard_normal((U, 16)), rng.standard_normal((I, 16))
    ch = Chain64(e, U, I, kind, cred)
    uf, itf, lu, li = ch.forward(u0, i0, K, order, keep_u=np.arange(U), keep_i=np.arange(I))
    gu, gi = ch.backward(u0, i0, K, order)
    if kind == "j":
        a, b, _ = R.j_mats(e, U, I, cred)
        ruf, ritf, us, is_ = R.propagate_j(a, b, u0, i0, K)
        rgu, rgi = R.backward_j(a, b, u0, i0, K)
    else:
        a, b = R.gs_mats(e, U, I, cred, method_a=kind == "method_a")
        ruf, ritf, us, is_ = R.propagate_gs(a, b, u0, i0, K)
        rgu, rgi = R.backward_gs(a, b, u0, i0, K)
    for got, want in [(uf, ruf), (itf, ritf), (gu, rgu), (gi, rgi)] + list(zip(lu, us)) \
            + list(zip(li, is_)):
        assert nrel(got, want) < 1e-13
