"""GPU: the drop-in step through the registered torch operators (ops.py).

The reference's step (Version-2/lighgcn_cu_pop.py:858-863):
    u_final, i_final = model.propagate()
    loss = model.bpr_loss(users, pos, neg, u_final, i_final, reg)
    opt.zero_grad(); loss.backward(); opt.step()
* under torch.compile (backend "aot_eager": dynamo + AOTAutograd trace the
  bbgr ops through their fake kernels and registered backward; no code
  generation) it gives the eager step's loss and gradients bit for bit;
* captured whole into a CUDA graph (forward, backward and a capturable
  torch.optim.Adam) and replayed, it gives the eager steps' weights bit for bit.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from bbgr import lightgcn as L  # noqa: E402
from bbgr import lightgcn_cu as J  # noqa: E402
from bbgr import lightgcn_cu_pop as V2  # noqa: E402
from bbgr.synthetic import synthetic_credibility, synthetic_edges  # noqa: E402

DEV = "cuda"
U, I, E, D, K, B = 1500, 700, 20000, 64, 3, 512


def _model(family, seed=0, layers=K):
    e = synthetic_edges(U, I, E, seed=4, items="zipf")
    torch.manual_seed(seed)
    if family == "v2":
        cred = torch.as_tensor(synthetic_credibility(U, 4))
        M_ui, M_iu = V2.build_message_passing_mats(e, U, I, cred, DEV)
        m = V2.LightGCN(U, I, D, layers, M_ui, M_iu).to(DEV)
    elif family == "cu":
        cred = torch.as_tensor(synthetic_credibility(U, 4))
        M_ui, M_iu, deg_i = J.build_cred_weighted_mats(e, U, I, cred, DEV)
        m = J.CredLightGCN(U, I, D, layers, M_ui, M_iu).to(DEV)
        m.pop = torch.as_tensor(deg_i / max(deg_i.max(), 1.0), device=DEV)
    else:
        A = L.build_norm_adj(e, U, I, DEV)
        m = L.LightGCN(U, I, D, layers, A).to(DEV)
    return m


def _batch(seed):
    """Random triples with repeated users and items: the BPR backward sums
    each row's addends in a fixed order (bbgr::bpr_loss_backward), so runs
    still compare bitwise."""
    g = torch.Generator().manual_seed(seed)
    users = torch.randint(0, U, (B,), generator=g).to(DEV)
    pos = torch.randint(0, I, (B,), generator=g).to(DEV)
    neg = torch.randint(0, I, (B,), generator=g).to(DEV)
    return users, pos, neg


def _loss(m, users, pos, neg):
    if isinstance(m, J.CredLightGCN):   # lightgcn_cu.py:583-584, 635-648
        uf, itf = m.final_embeddings()
        return m.bpr_fair_loss(users, pos, neg, uf, itf, m.pop, 0.05, 1e-4)
    uf, itf = m.get_user_item_emb()
    return m.bpr_loss(users, pos, neg, uf, itf, 1e-4)


def test_per_layer_op_matches_fused_propagation():
    """propagate_all_layers (one bbgr::jacobi_layer per layer) -> layer mean
    equals final_embeddings (bbgr::propagate) to fp32 rounding, forward and
    gradient."""
    m = _model("cu")
    us, is_ = m.propagate_all_layers()
    uf = torch.stack(us).mean(0)
    itf = torch.stack(is_).mean(0)
    ufr, itfr = m.final_embeddings()
    for a, b in ((uf, ufr), (itf, itfr)):
        assert float((a - b).norm() / b.norm()) < 1e-6
    (uf.sum() + 2 * itf.sum()).backward()
    g1 = [p.grad.clone() for p in m.parameters()]
    m.zero_grad()
    (ufr.sum() + 2 * itfr.sum()).backward()
    for a, p in zip(g1, m.parameters()):
        assert float((a - p.grad).norm() / p.grad.norm()) < 1e-6


@pytest.mark.parametrize("family", ["v2", "cu", "sym"])
def test_compiled_step_matches_eager(family):
    a, b = _model(family), _model(family)
    users, pos, neg = _batch(1)
    la = _loss(a, users, pos, neg)
    la.backward()
    _loss(b, users, pos, neg)          # resolves the operator pair outside the trace
    b.zero_grad()
    step = torch.compile(_loss, backend="aot_eager", fullgraph=False)
    lb = step(b, users, pos, neg)
    lb.backward()
    assert float(la) == float(lb)
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.equal(pa.grad, pb.grad)


@pytest.mark.parametrize("family", ["v2", "sym"])
def test_cuda_graph_captured_step_matches_eager(family):
    """Whole drop-in step (forward, backward, Adam) captured once, replayed on
    new batches copied into static buffers: weights equal the eager run."""
    a, b = _model(family), _model(family)
    oa = torch.optim.Adam(a.parameters(), lr=1e-3, capturable=True)
    ob = torch.optim.Adam(b.parameters(), lr=1e-3, capturable=True)
    batches = [_batch(s) for s in range(6)]

    def eager_step(m, opt, bt):
        loss = _loss(m, *bt)
        opt.zero_grad(set_to_none=False)
        loss.backward()
        opt.step()
        return loss

    for bt in batches:
        eager_step(a, oa, bt)
    # b: two warm-up steps on a side stream, capture, replay the rest
    static = [t.clone() for t in batches[0]]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for bt in batches[:2]:
            for dst, src in zip(static, bt):
                dst.copy_(src)
            eager_step(b, ob, static)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        static_loss = eager_step(b, ob, static)
    for bt in batches[2:]:
        for dst, src in zip(static, bt):
            dst.copy_(src)
        graph.replay()
    torch.cuda.synchronize()
    assert np.isfinite(float(static_loss))
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.equal(pa, pb)


@pytest.mark.parametrize("d,ld", [(64, 64), (8, 8), (32, 64), (256, 256), (12, 13)])
def test_row_support_kernel(d, ld):
    """bbgr_row_support: nonzero rows flagged (-0.0 is zero), every other row
    cleared, and with a CSR every neighbour of a flagged row set."""
    import ctypes  # noqa: F401
    from bbgr._lib import call, ld as ld_, ptr, stream_handle
    n, m = 3000, 500
    g = torch.Generator().manual_seed(d)
    x = torch.zeros(n, ld)
    live = torch.randperm(n, generator=g)[:200]
    x[live, torch.randint(0, d, (200,), generator=g)] = torch.randn(200, generator=g)
    x[torch.randperm(n, generator=g)[:50], 0] = -0.0
    if ld > d:   # junk beyond the row's d columns must not count
        x[:, d:] = 7.0
    x = x.to(DEV)
    xs = x[:, :d] if ld > d else x
    e = torch.stack([torch.randint(0, n, (20000,), generator=g),
                     torch.randint(0, m, (20000,), generator=g)])
    order = torch.argsort(e[0] * m + e[1])
    rows, cols = e[0][order], e[1][order]
    indptr = torch.zeros(n + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(torch.bincount(rows, minlength=n), 0)
    indptr_d = indptr.to(torch.int32).to(DEV)
    cols_d = cols.to(torch.int32).to(DEV)
    mask = torch.full((n,), 9, dtype=torch.uint8, device=DEV)
    nbr = torch.zeros(m, dtype=torch.uint8, device=DEV)
    call("bbgr_row_support", n, d, ptr(xs), ld_(xs), ptr(mask), ptr(indptr_d), ptr(cols_d),
         ptr(nbr), stream_handle())
    want = (x[:, :d].cpu() != 0).any(1)
    assert torch.equal(mask.cpu().bool(), want) and int(mask.max()) <= 1
    want_nbr = torch.zeros(m, dtype=torch.bool)
    sel = want[rows]
    want_nbr[cols[sel]] = True
    assert torch.equal(nbr.cpu().bool(), want_nbr)


@pytest.mark.parametrize("family", ["v2", "cu", "sym"])
def test_cpp_operators_equal_the_python_chain(family):
    """torch.ops.bbgr.* (csrc/torch_ops.cpp) issue the same launches as the
    Python chain (propagate.forward / backward): bitwise equal outputs."""
    from bbgr import ops
    from bbgr.propagate import ORDER_GS, ORDER_J, backward, forward
    m = _model(family)
    pair = m.norm_adj.pair if family == "sym" else m._operator_pair()
    order = ORDER_GS if family == "v2" else ORDER_J
    if family == "sym":
        u0, i0 = m.emb.weight[:U].detach(), m.emb.weight[U:].detach()
    else:
        u0, i0 = m.user_emb.weight.detach(), m.item_emb.weight.detach()
    key = ops.pair_key(pair)
    a = ops.propagate(u0, i0, key, K, order)
    b = forward(pair, u0, i0, K, order)
    assert all(torch.equal(x, y) for x, y in zip(a, b))
    g = torch.Generator().manual_seed(9)
    gU, gI = torch.randn(U, D, generator=g).to(DEV), torch.randn(I, D, generator=g).to(DEV)
    a = ops.propagate_backward(gU, gI, key, K, order)
    b = backward(pair, gU, gI, K, order)
    assert all(torch.equal(x, y) for x, y in zip(a, b))
    if family == "sym":
        x0 = m.emb.weight.detach()
        assert torch.equal(ops.propagate_sym(x0, key, K), torch.cat(forward(pair, u0, i0, K,
                                                                           ORDER_J)))


@pytest.mark.parametrize("order", ["gs", "jacobi"])
def test_backward_op_support_masks_are_bitwise_dense(order):
    """bbgr::propagate_backward reads the gradients' row support and masks the
    first backward products: bitwise the unmasked (dense) chain on a BPR-shaped
    gradient (batch rows only)."""
    from bbgr import ops
    from bbgr.propagate import backward
    m = _model("v2")
    pair = m._operator_pair()
    users, pos, neg = _batch(3)
    gU = torch.zeros(U, D, device=DEV)
    gI = torch.zeros(I, D, device=DEV)
    gU[users] = torch.randn(B, D, device=DEV)
    gI[torch.cat([pos, neg])] = torch.randn(2 * B, D, device=DEV)
    a_u, a_i = ops.propagate_backward(gU, gI, ops.pair_key(pair), K, order)
    b_u, b_i = backward(pair, gU, gI, K, order)
    assert torch.equal(a_u, b_u) and torch.equal(a_i, b_i)


@pytest.mark.parametrize("family,layers", [("v2", K), ("cu", K), ("v2", 0), ("cu", 0)])
def test_sparse_ego_gradient_is_bitwise_dense(family, layers, monkeypatch):
    """Eager drop-in step: bpr_loss picks bbgr::bpr_loss_sparse_ego (the final
    tables come from the propagate op, which returns dense gradients for the
    same weights), whose backward hands the ego gradient and dL/d(u_final) back
    as sparse rows (propagate_backward_rows); .grad stays dense and equals the
    dense op's bit for bit, with repeated users / items and a dropped triple
    (neg = -1). K = 0 (the reference's layer loop runs zero times) included:
    grad_u0 is then gU itself, every row of it."""
    from bbgr import bpr, ops
    users, pos, neg = _batch(5)
    neg = neg.clone()
    neg[7] = -1
    grads = {}
    for mode in ("sparse", "dense"):
        if mode == "dense":
            monkeypatch.setattr(bpr, "_receives_dense_grad", lambda *a: False)
        m = _model(family, layers=layers)
        loss = _loss(m, users, pos, neg)
        assert ("sparseego" in loss.grad_fn.name().lower()) == (mode == "sparse")
        n0 = ops.counters()
        loss.backward()
        n1 = ops.counters()
        # sparse mode: dL/d(u_final) reaches propagate's backward as rows too
        assert n1["rows"] - n0["rows"] == (1 if mode == "sparse" else 0)
        assert n1["dense"] - n0["dense"] == (0 if mode == "sparse" else 1)
        grads[mode] = (float(loss), [p.grad for p in m.parameters()])
        assert all(p.grad.layout == torch.strided for p in m.parameters())
    assert grads["sparse"][0] == grads["dense"][0]
    for a, b in zip(grads["sparse"][1], grads["dense"][1]):
        assert torch.equal(a, b)


def test_sparse_ego_not_chosen_without_dense_path():
    """bpr_loss on tables that do not come from the propagate node keeps the
    dense ego gradient (so .grad never turns sparse)."""
    m = _model("v2")
    uf, itf = m.get_user_item_emb()
    users, pos, neg = _batch(6)
    loss = m.bpr_loss(users, pos, neg, uf.detach(), itf.detach(), 1e-4)
    assert "sparse" not in loss.grad_fn.name().lower()
    loss.backward()
    assert m.user_emb.weight.grad.layout == torch.strided
    # a node with a direct edge to the weight that is NOT the propagate op (an
    # Add here; an nn.Embedding(sparse=True) lookup alike) keeps the dense form
    m.zero_grad()
    uf2 = m.user_emb.weight + uf.detach()
    itf2 = m.item_emb.weight + itf.detach()
    loss = m.bpr_loss(users, pos, neg, uf2, itf2, 1e-4)
    assert "sparse" not in loss.grad_fn.name().lower()
    loss.backward()
    assert m.user_emb.weight.grad.layout == torch.strided


@pytest.mark.parametrize("order", ["degree", "input"])
@pytest.mark.parametrize("d", [64, 128])
def test_dropin_first_item_product_bitmap_is_bitwise_the_mask(order, d, monkeypatch):
    """GS rows backward (bbgr::propagate_backward_rows): the first backward
    item product visits the item frontier as a device-length row list and
    tests edge liveness on the slot bitmap of the batch users' edges in
    item-CSR order (frontier_bits / u2i_slots in csrc/torch_ops.cpp). The loss
    and both weight gradients equal the mask-only product's
    (BBGR_DROPIN_BITS=0) bit for bit, on a Zipf graph whose hub items are cut
    into one chunk and into several, with duplicate edges, in both drop-in
    vertex orders."""
    from bbgr import operators, ops
    U_, I_, E_, B_ = 20000, 1500, 400_000, 1024
    e = synthetic_edges(U_, I_, E_, seed=7, items="zipf", duplicates=50)
    deg_i = np.bincount(np.asarray(e)[1], minlength=I_)
    assert (deg_i > 2048).sum() >= 3 and ((deg_i > 256) & (deg_i <= 2048)).sum() >= 10
    cred = torch.as_tensor(synthetic_credibility(U_, 5))
    g = torch.Generator().manual_seed(3)
    users = torch.randint(0, U_, (B_,), generator=g).to(DEV)
    pos = torch.randint(0, I_, (B_,), generator=g).to(DEV)
    neg = torch.randint(0, I_, (B_,), generator=g).to(DEV)
    monkeypatch.setattr(operators, "DROPIN_VERTEX_ORDER", order)
    M_ui, M_iu = V2.build_message_passing_mats(e, U_, I_, cred, DEV)
    out = {}
    # (BBGR_MASK_BITS: the first user product's per-edge test on the packed
    # item mask, bbgr_mask_pack, vs the bytes; also bitwise)
    for bits, mb in (("1", "1"), ("1", "0"), ("0", "0")):
        monkeypatch.setenv("BBGR_DROPIN_BITS", bits)
        monkeypatch.setenv("BBGR_MASK_BITS", mb)
        torch.manual_seed(0)
        m = V2.LightGCN(U_, I_, d, K, M_ui, M_iu).to(DEV)
        uf, itf = m.propagate()
        loss = m.bpr_loss(users, pos, neg, uf, itf, 1e-4)
        n0 = ops.counters()
        loss.backward()
        assert ops.counters()["rows"] - n0["rows"] == 1
        out[bits + mb] = (float(loss), [p.grad.clone() for p in m.parameters()])
    for key in ("10", "00"):
        assert out["11"][0] == out[key][0]
        for a, b in zip(out["11"][1], out[key][1]):
            assert torch.equal(a, b)
