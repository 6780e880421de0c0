"""GPU: the reference's training loops, end to end, over several steps.

Each family's loop — Version-2/lighgcn_cu_pop.py:786-863 (GS, pop-mix
negatives), version_1/lightgcn_cu_pop_long_tail_exposure.py:630-685 (Method
A: popularity-damped GS, uniform negatives), lightgcn_cu.py:586-652 (Jacobi,
uniform negatives, the credibility-fair loss written inline) and
lightgcn.py:540-590 (symmetric adjacency, uniform negatives): the operators, the model, torch's Adam, the
seeded numpy stream, the per-epoch shuffle of the train users, the per-user
sampler loop and the step — runs twice on the C1 graph:

(a) restated on the CPU: oracle/ref_numpy (CSR, popularity, the sampler
    loops) and oracle/ref_torch (fp32 torch.sparse operators and models,
    torch.optim.Adam) — the checker;
(b) through this repo's boundary: bbgr.host_sampler with its own Generator
    and the family's drop-in module on the GPU (for Version-2 also with
    bbgr.optim.FusedAdam(fuse_backward=True)).

The samples are integers and must be identical, and both Generators end in
the same state. Per-step losses agree to 1e-5 relative, the weights after the
last step to 1e-4 normwise and the training updates (weights minus the
initial ones) to 1e-2 normwise: Adam's early steps move each weight by about
lr * sign(g), so fp32 rounding of a near-zero gradient component can flip a
few of them.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from bbgr import host_sampler as HS  # noqa: E402
from bbgr import lightgcn as SYM  # noqa: E402
from bbgr import lightgcn_cu as CU  # noqa: E402
from bbgr import lightgcn_cu_pop as V2  # noqa: E402
from bbgr import lightgcn_cu_pop_long_tail_exposure as MA  # noqa: E402
from bbgr.synthetic import CONFIGS, config_edges, synthetic_credibility  # noqa: E402
from oracle import ref_numpy as R  # noqa: E402
from oracle import ref_torch as T  # noqa: E402

DEV = "cuda"
LAMBDA_FAIR = 0.01


def _pop_prob(edges, num_items, gamma=0.75):
    """The caller's popularity vector, written as the loop writes it
    (Version-2/lighgcn_cu_pop.py:805-810)."""
    deg = np.bincount(edges[1].astype(np.int64), minlength=num_items).astype(np.float64)
    pop = np.power(deg + 1.0, gamma)
    return (pop / (pop.sum() + 1e-12)).astype(np.float64)


def _v2(e, U, I, d, K, cred, optimizer, lr):
    torch.manual_seed(42)
    Tui, Tiu = T.gs_operators(e, U, I, cred)
    ref = T.GSModel(U, I, d, K, Tui, Tiu)
    M_ui, M_iu = V2.build_message_passing_mats(e, U, I, torch.as_tensor(cred), DEV)
    m = V2.LightGCN(U, I, d, K, M_ui, M_iu).to(DEV)
    tables = {"user_emb": (m.user_emb, ref.user_emb), "item_emb": (m.item_emb, ref.item_emb)}

    def step(users_t, pos_t, neg_t, reg):   # Version-2/lighgcn_cu_pop.py:858-859
        user_emb, item_emb = m.get_user_item_emb()
        return m.bpr_loss(users_t, pos_t, neg_t, user_emb, item_emb, reg)

    if optimizer == "fused_backward":
        from bbgr.optim import FusedAdam
        return ref, m, tables, step, lambda ps: FusedAdam(ps, lr=lr, fuse_backward=True)
    return ref, m, tables, step, None


def _method_a(e, U, I, d, K, cred, optimizer, lr):
    """version_1/lightgcn_cu_pop_long_tail_exposure.py:630-685: Version-2's
    model on the popularity-damped operators, uniform negatives."""
    torch.manual_seed(42)
    Tui, Tiu = T.gs_operators(e, U, I, cred, method_a=True)
    ref = T.GSModel(U, I, d, K, Tui, Tiu)
    M_ui, M_iu = MA.build_message_passing_mats(e, U, I, torch.as_tensor(cred), DEV)
    m = MA.LightGCN(U, I, d, K, M_ui, M_iu).to(DEV)
    tables = {"user_emb": (m.user_emb, ref.user_emb), "item_emb": (m.item_emb, ref.item_emb)}

    def step(users_t, pos_t, neg_t, reg):
        user_emb, item_emb = m.get_user_item_emb()
        return m.bpr_loss(users_t, pos_t, neg_t, user_emb, item_emb, reg)

    return ref, m, tables, step, None


def _cu(e, U, I, d, K, cred, optimizer, lr):
    torch.manual_seed(42)
    ref, _ = T.reference_model("cu_fair", e, U, I, d, K, cred, lambda_fair=LAMBDA_FAIR)
    M_ui, M_iu, deg_i = CU.build_cred_weighted_mats(e, U, I, cred, DEV)
    pop_t = torch.tensor((deg_i / max(float(deg_i.max()), 1.0)).astype(np.float32), device=DEV)
    m = CU.CredLightGCN(U, I, d, K, M_ui, M_iu).to(DEV)
    tables = {"user_emb": (m.user_emb, ref.user_emb), "item_emb": (m.item_emb, ref.item_emb)}

    def step(users_t, pos_t, neg_t, reg):   # lightgcn_cu.py:632-648, as written there
        e_u, e_i = m.final_embeddings()
        pos_scores = m.score(users_t, pos_t, e_u, e_i)
        neg_scores = m.score(users_t, neg_t, e_u, e_i)
        loss_bpr = -torch.log(torch.sigmoid(pos_scores - neg_scores) + 1e-12).mean()
        loss_fair = (pop_t[pos_t] * pos_scores).mean()
        loss_reg = m.l2_reg(users_t, pos_t, neg_t)
        return loss_bpr + LAMBDA_FAIR * loss_fair + reg * loss_reg

    return ref, m, tables, step, None


def _sym(e, U, I, d, K, cred, optimizer, lr):
    torch.manual_seed(42)
    ref = T.SymModel(U, I, d, K, T.sym_operator(e, U, I))
    m = SYM.LightGCN(U, I, d, K, SYM.build_norm_adj(e, U, I, DEV)).to(DEV)
    tables = {"emb": (m.emb, ref.emb)}

    def step(users_t, pos_t, neg_t, reg):   # lightgcn.py:584-585
        user_emb, item_emb = m.get_user_item_emb()
        return m.bpr_loss(users_t, pos_t, neg_t, user_emb, item_emb, reg)

    return ref, m, tables, step, None


FAMILIES = {"v2_pop": (_v2, True), "method_a": (_method_a, False), "cu_fair": (_cu, False),
            "plain": (_sym, False)}


@pytest.mark.parametrize("family,optimizer", [("v2_pop", "torch"), ("v2_pop", "fused_backward"),
                                              ("method_a", "torch"), ("cu_fair", "torch"),
                                              ("plain", "torch")])
def test_reference_training_loop_two_epochs(family, optimizer):
    c = CONFIGS["C1"]
    U, I, d, K = c["num_users"], c["num_items"], c["emb_dim"], c["num_layers"]
    B, epochs, reg, lr = 256, 2, 1e-4, 1e-3
    e = config_edges("C1")
    cred = synthetic_credibility(U, 7)
    make, popmix = FAMILIES[family]
    ref, m, tables, step, make_opt = make(e, U, I, d, K, cred, optimizer, lr)

    # (a) the restated reference's loop state
    ropt = torch.optim.Adam(ref.parameters(), lr=lr)
    r_ptr, r_idx = R.edges_to_user_csr(e, U)
    r_pop = R.pop_prob(e, I) if popmix else None
    r_rng = np.random.default_rng(42)
    r_users = np.where(np.diff(r_ptr) > 0)[0]

    # (b) the drop-in's, from the same initial weights
    w0 = {n: rt.weight.detach().clone().double() for n, (_, rt) in tables.items()}
    with torch.no_grad():
        for mt, rt in tables.values():
            mt.weight.copy_(rt.weight)
    opt = make_opt(m.parameters()) if make_opt else torch.optim.Adam(m.parameters(), lr=lr)
    o_ptr, o_idx = HS.edges_to_user_csr(e, U)
    o_pop = _pop_prob(e, I) if popmix else None
    o_rng = np.random.default_rng(42)
    o_users = np.where(np.diff(o_ptr) > 0)[0]
    assert np.array_equal(o_ptr, r_ptr) and np.array_equal(o_idx, r_idx)

    steps = 0
    for _ in range(epochs):
        r_rng.shuffle(r_users)
        o_rng.shuffle(o_users)
        assert np.array_equal(o_users, r_users)
        for start in range(0, len(r_users), B):
            rb, ob = r_users[start:start + B], o_users[start:start + B]
            if popmix:
                ru, rp, rn = R.sample_batch_reference_style(r_ptr, r_idx, rb, I, r_rng, r_pop)
            else:
                ru, rp, rn = R.sample_batch_uniform_reference_style(r_ptr, r_idx, rb, I, r_rng)
            ou, op, on = HS.sample_batch(o_ptr, o_idx, ob, I, o_rng, o_pop)
            assert all(np.array_equal(x, y) for x, y in ((ou, ru), (op, rp), (on, rn)))
            rloss = T.train_step(ref, ropt, torch.as_tensor(ru), torch.as_tensor(rp),
                                 torch.as_tensor(rn), reg)
            users_t, pos_t, neg_t = (torch.tensor(x, device=DEV, dtype=torch.long)
                                     for x in (ou, op, on))
            loss = step(users_t, pos_t, neg_t, reg)
            opt.zero_grad()
            loss.backward()
            opt.step()
            assert abs(float(loss) - rloss) <= 1e-5 * rloss, (steps, float(loss), rloss)
            steps += 1
    assert steps == epochs * ((len(r_users) + B - 1) // B)
    assert r_rng.bit_generator.state == o_rng.bit_generator.state
    for name, (mt, rt) in tables.items():
        w = mt.weight.detach().cpu().double()
        rw = rt.weight.detach().double()
        assert float((w - rw).norm() / rw.norm()) < 1e-4, name
        # the training updates themselves, normwise
        dw, drw = w - w0[name], rw - w0[name]
        assert float((dw - drw).norm() / drw.norm()) < 1e-2, name
