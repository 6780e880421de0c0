"""GPU: the reference's training loop, end to end, over several steps.

Version-2/lighgcn_cu_pop.py:786-863 — the operators, the model, the
optimizer, the seeded numpy stream, the per-epoch shuffle of the train users,
the per-user pop-mix sampler loop and the step — run twice on one C1-sized
synthetic graph:

(a) restated on the CPU: oracle/ref_numpy (CSR, popularity, the sampler loop)
    and oracle/ref_torch (fp32 torch.sparse operators, the GS model,
    torch.optim.Adam) — the checker;
(b) through this repo's boundary: bbgr.host_sampler with its own Generator,
    bbgr.lightgcn_cu_pop on the GPU, with torch's Adam or with
    bbgr.optim.FusedAdam(fuse_backward=True).

The samples are integers and must be identical; the per-step losses agree to
1e-5 relative, the weights after the last step to 1e-4 normwise and the
training updates (weights minus the initial ones) to 1e-2 normwise (Adam's
early steps move each weight by about lr * sign(g), so fp32 rounding of a
near-zero gradient component can flip a few of them).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from bbgr import host_sampler as HS  # noqa: E402
from bbgr import lightgcn_cu_pop as V2  # noqa: E402
from bbgr.synthetic import CONFIGS, config_edges, synthetic_credibility  # noqa: E402
from oracle import ref_numpy as R  # noqa: E402
from oracle import ref_torch as T  # noqa: E402

DEV = "cuda"


def _pop_prob(edges, num_items, gamma=0.75):
    """The caller's popularity vector, written as the loop writes it
    (Version-2/lighgcn_cu_pop.py:805-810)."""
    deg = np.bincount(edges[1].astype(np.int64), minlength=num_items).astype(np.float64)
    pop = np.power(deg + 1.0, gamma)
    return (pop / (pop.sum() + 1e-12)).astype(np.float64)


@pytest.mark.parametrize("optimizer", ["torch", "fused_backward"])
def test_reference_training_loop_two_epochs(optimizer):
    c = CONFIGS["C1"]
    U, I, d, K = c["num_users"], c["num_items"], c["emb_dim"], c["num_layers"]
    B, epochs, reg, lr = 256, 2, 1e-4, 1e-3
    e = config_edges("C1")
    cred = synthetic_credibility(U, 7)

    # (a) the restated reference
    torch.manual_seed(42)
    Tui, Tiu = T.gs_operators(e, U, I, cred)
    ref = T.GSModel(U, I, d, K, Tui, Tiu)
    ropt = torch.optim.Adam(ref.parameters(), lr=lr)
    r_ptr, r_idx = R.edges_to_user_csr(e, U)
    r_pop = R.pop_prob(e, I)
    r_rng = np.random.default_rng(42)
    r_users = np.where(np.diff(r_ptr) > 0)[0]

    # (b) the drop-in, from the same initial weights
    M_ui, M_iu = V2.build_message_passing_mats(e, U, I, torch.as_tensor(cred), DEV)
    m = V2.LightGCN(U, I, d, K, M_ui, M_iu).to(DEV)
    w0 = {n: getattr(ref, n).weight.detach().clone().double() for n in ("user_emb", "item_emb")}
    with torch.no_grad():
        m.user_emb.weight.copy_(ref.user_emb.weight)
        m.item_emb.weight.copy_(ref.item_emb.weight)
    if optimizer == "torch":
        opt = torch.optim.Adam(m.parameters(), lr=lr)
    else:
        from bbgr.optim import FusedAdam
        opt = FusedAdam(m.parameters(), lr=lr, fuse_backward=True)
    o_ptr, o_idx = HS.edges_to_user_csr(e, U)
    o_pop = _pop_prob(e, I)
    o_rng = np.random.default_rng(42)
    o_users = np.where(np.diff(o_ptr) > 0)[0]
    assert np.array_equal(o_ptr, r_ptr) and np.array_equal(o_idx, r_idx)

    steps = 0
    for _ in range(epochs):
        r_rng.shuffle(r_users)
        o_rng.shuffle(o_users)
        assert np.array_equal(o_users, r_users)
        for start in range(0, len(r_users), B):
            ru, rp, rn = R.sample_batch_reference_style(r_ptr, r_idx, r_users[start:start + B], I,
                                                        r_rng, r_pop)
            ou, op, on = HS.sample_batch(o_ptr, o_idx, o_users[start:start + B], I, o_rng, o_pop)
            assert all(np.array_equal(x, y) for x, y in ((ou, ru), (op, rp), (on, rn)))
            rloss = T.train_step(ref, ropt, torch.as_tensor(ru), torch.as_tensor(rp),
                                 torch.as_tensor(rn), reg)
            users_t, pos_t, neg_t = (torch.tensor(x, device=DEV, dtype=torch.long)
                                     for x in (ou, op, on))
            user_emb, item_emb = m.get_user_item_emb()
            loss = m.bpr_loss(users_t, pos_t, neg_t, user_emb, item_emb, reg)
            opt.zero_grad()
            loss.backward()
            opt.step()
            assert abs(float(loss) - rloss) <= 1e-5 * rloss, (steps, float(loss), rloss)
            steps += 1
    assert steps == epochs * ((len(r_users) + B - 1) // B)
    assert r_rng.bit_generator.state == o_rng.bit_generator.state
    for name in ("user_emb", "item_emb"):
        w = getattr(m, name).weight.detach().cpu().double()
        rw = getattr(ref, name).weight.detach().double()
        assert float((w - rw).norm() / rw.norm()) < 1e-4, name
        # the training updates themselves, normwise
        dw, drw = w - w0[name], rw - w0[name]
        assert float((dw - drw).norm() / drw.norm()) < 1e-2, name
