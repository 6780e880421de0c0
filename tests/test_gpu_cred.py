"""GPU: credibility-GNN aggregation (main.py:645-707) vs the oracle
restatements (oracle/ref_numpy float64, oracle/ref_torch.CredModelRef fp32 CPU)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import ref_numpy as R  # noqa: E402

DEV = "cuda"


def _subgraph(nu, ni, E, seed, hub=True):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, nu, E)
    dst = rng.integers(0, ni - 1, E)              # item ni-1 stays isolated
    if hub:                                        # a destination with > 256 edges (chunked rows)
        src = np.concatenate([src, rng.integers(0, nu, 3000)])
        dst = np.concatenate([dst, np.zeros(3000, np.int64)])
    src = np.concatenate([src, src[:20]])          # duplicate edges
    dst = np.concatenate([dst, dst[:20]])
    ea = rng.uniform(-0.5, 1.5, (src.size, 5)).astype(np.float32)
    ea[:50, 0] = 0.0
    ea[:50, 1] = -1.0                              # zero-weight edges (clamp(min=0))
    return np.stack([src, dst]), ea


def _close(got, want, what, tol=1e-5):
    got = got.detach().double().cpu().numpy()
    want = np.asarray(want, np.float64)
    err = np.linalg.norm(got - want) / max(np.linalg.norm(want), 1e-30)
    assert err <= tol and np.abs(got - want).max() <= tol * max(np.abs(want).max(), 1e-30), \
        (what, err)


def test_edge_weights_and_aggregation_vs_oracle():
    from bbgr.cred_gnn import EdgeSet, aggregate
    nu, ni = 900, 400
    ei, ea = _subgraph(nu, ni, 20000, 1)
    es = EdgeSet(torch.tensor(ei, device=DEV), nu, ni)
    w_raw, w_t, w_c = es.normalize(edge_attr=torch.tensor(ea, device=DEV))
    want_raw = R.ewa_raw(ea)
    np.testing.assert_array_equal(w_raw.cpu().numpy(), want_raw)       # elementwise, exact
    want_t = R.normalize_per_dst(want_raw, ei[1], ni)
    _close(w_t, want_t, "w_tilde", 1e-6)
    x = torch.randn(nu, 64, device=DEV)
    x.requires_grad_(True)
    out = aggregate(x, es, w_t, w_c)
    _close(out, R.aggregate(x.detach().cpu().numpy(), ei, want_t, ni), "aggregate")
    assert out[ni - 1].abs().sum().item() == 0
    g = torch.randn(ni, 64, device=DEV)
    (out * g).sum().backward()
    want_gx = R.aggregate(g.cpu().numpy(), ei[::-1], want_t, nu)      # transpose
    _close(x.grad, want_gx, "d aggregate / d x")
    out2 = aggregate(x.detach(), es, w_t, w_c)
    assert torch.equal(out.detach(), out2)                           # deterministic


def test_reference_methods_individually():
    from bbgr.cred_gnn import CredModel
    nu, ni = 300, 200
    ei, ea = _subgraph(nu, ni, 5000, 2, hub=False)
    m = CredModel(8, 6, 64).to(DEV)
    w = m.ewa_raw(torch.tensor(ea, device=DEV))
    np.testing.assert_array_equal(w.cpu().numpy(), R.ewa_raw(ea))
    wt = m.normalize_per_dst(w, torch.tensor(ei[1], device=DEV), ni)
    _close(wt, R.normalize_per_dst(R.ewa_raw(ea), ei[1], ni), "normalize_per_dst", 1e-6)
    x = torch.randn(nu, 64, device=DEV)
    out = m.aggregate(x, torch.tensor(ei, device=DEV), wt, ni)
    _close(out, R.aggregate(x.cpu().numpy(), ei, wt.cpu().numpy(), ni), "aggregate")


@pytest.mark.parametrize("hidden", [64, 128])
def test_cred_model_forward_backward_vs_torch_reference(hidden):
    """Whole forward_subgraph + BCE/smoothness loss backward: device model vs
    the fp32 torch CPU restatement with identical weights."""
    from bbgr.cred_gnn import CredModel
    from oracle.ref_torch import CredModelRef
    torch.manual_seed(0)
    nu, ni = 1200, 500
    ei, ea = _subgraph(nu, ni, 15000, 3)
    x_u = torch.randn(nu, 9)
    x_i = torch.randn(ni, 7)
    ref = CredModelRef(9, 7, hidden)
    dev = CredModel(9, 7, hidden).to(DEV)
    dev.load_state_dict({k: v.to(DEV) for k, v in ref.state_dict().items()})
    e_u2i = torch.tensor(ei)
    e_i2u = torch.stack([e_u2i[1], e_u2i[0]])
    eat = torch.tensor(ea)
    outs_r = ref.forward_subgraph(x_u, x_i, e_u2i, eat, e_i2u, eat)
    outs_d = dev.forward_subgraph(x_u.to(DEV), x_i.to(DEV), e_u2i.to(DEV), eat.to(DEV),
                                  e_i2u.to(DEV), eat.to(DEV))
    for a, b, what in zip(outs_d, outs_r, ("cred", "h_u2", "h_i1", "w1t")):
        _close(a, b.detach().numpy(), what, 2e-5)
    y = (torch.rand(nu) > 0.5).float()

    def loss_of(outs, yy):
        cred, h_u2, h_i1, w1t = outs
        return F_bce(cred, yy) + 0.1 * (w1t * (h_u2[e_u2i[0].to(cred.device)] -
                                               h_i1[e_u2i[1].to(cred.device)]).pow(2).sum(-1)).mean()

    F_bce = torch.nn.functional.binary_cross_entropy
    loss_of(outs_r, y).backward()
    loss_of(outs_d, y.to(DEV)).backward()
    for (n, p_r), (_, p_d) in zip(ref.named_parameters(), dev.named_parameters()):
        _close(p_d.grad, p_r.grad.numpy(), f"grad {n}", 1e-4)


@pytest.mark.parametrize("given_w", [False, True])
def test_normalize_with_and_without_dst_is_bitwise_equal(given_w):
    """bbgr_ewa_normalize writes w~ in input order either by a coalesced pass
    over the edges (dst given, what EdgeSet does) or by the scatter through the
    CSR permutation (dst NULL): the same values, bit for bit."""
    import ctypes
    from bbgr._lib import call, ptr, stream_handle
    from bbgr.cred_gnn import EdgeSet
    nu, ni = 700, 300
    ei, ea = _subgraph(nu, ni, 12000, 5)
    es = EdgeSet(torch.tensor(ei, device=DEV), nu, ni)
    E = es.E
    attr = torch.tensor(ea, device=DEV)
    w_in = torch.rand(E, device=DEV) if given_w else None
    outs = []
    for dst in (es.dst, None):
        w_raw, w_edge, w_csr = (torch.full((E,), -1.0, device=DEV) for _ in range(3))
        cs = es.by_dst.struct()
        args = (ctypes.byref(cs), ptr(es.by_dst.perm), ptr(dst), ptr(w_in),
                ptr(None if given_w else attr), 0 if given_w else attr.shape[1], 0, 1, 1.0, 1.0,
                1e-12, ptr(None if given_w else w_raw), ptr(w_edge), ptr(w_csr))
        n = ctypes.c_size_t(0)
        call("bbgr_ewa_normalize", *args, None, ctypes.byref(n), stream_handle())
        ws = torch.empty(max(n.value, 1), dtype=torch.uint8, device=DEV)
        call("bbgr_ewa_normalize", *args, ptr(ws), ctypes.byref(n), stream_handle())
        outs.append((w_edge, w_csr))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    raw = w_in.cpu().numpy() if given_w else R.ewa_raw(ea)
    _close(outs[0][0], R.normalize_per_dst(raw, ei[1], ni), "w_tilde", 1e-6)
