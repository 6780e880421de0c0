"""GPU: sampled evaluation (bbgr_eval_sampled) vs the oracle restatement of
Version-2/lighgcn_cu_pop.py:536-650 on the SAME candidates.

The native evaluate_sampled draws its candidates from the device Philox
stream, so those tests (1) check every candidate invariant exactly and (2) feed
the device's candidates to the float64 oracle and compare the metrics (fp32 vs
float64 scores can swap a near-tie, so per-user hit metrics may differ for at
most 2 users). The reference-signature wrappers draw the reference's own
numpy stream on the host (bbgr_eval_draw_candidates): their results are
checked against the whole reference loop, sampling included
(test_reference_signature_evaluation_is_the_reference_loop)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from bbgr.graph import Csr  # noqa: E402
from bbgr.synthetic import synthetic_credibility, synthetic_edges  # noqa: E402
from oracle import ref_numpy as R  # noqa: E402

DEV = "cuda"


def _split(U, I, E, seed):
    e = synthetic_edges(U, I, E, seed, items="zipf")
    rng = np.random.default_rng(seed)
    test = rng.random(e.shape[1]) < 0.2
    return e[:, ~test], e[:, test]


@pytest.mark.parametrize("d", [64, 128])
def test_eval_sampled_vs_oracle(d):
    from bbgr.evaluation import evaluate_sampled
    U, I = 2000, 1500
    tr, te = _split(U, I, 40000, 3)
    trc = Csr(tr[0], tr[1], U, I, DEV)
    tec = Csr(te[0], te[1], U, I, DEV)
    rng = np.random.default_rng(4)
    uf = rng.normal(size=(U, d)).astype(np.float32)
    itf = rng.normal(size=(I, d)).astype(np.float32)
    pop = np.bincount(tr[1], minlength=I)
    cred = synthetic_credibility(U, 3)
    res = evaluate_sampled(torch.tensor(uf, device=DEV), torch.tensor(itf, device=DEV), trc,
                           tec, I, pop, int(tr.shape[1]), cred, Ks=(10, 20), return_raw=True)
    raw = res.pop("_raw")
    users = raw["users"].cpu().numpy()
    cand = raw["cand"].cpu().numpy()
    assert raw["fails"] == 0
    tr_ptr, tr_idx = R.edges_to_user_csr(tr, U)
    te_ptr, te_idx = R.edges_to_user_csr(te, U)
    assert (np.diff(te_ptr)[users] > 0).all() and users.size == (np.diff(te_ptr) > 0).sum()
    for u, c in zip(users, cand):
        assert R.user_has_item(te_ptr, te_idx, u, c[0])               # pos from the test row
        for j in c[1:]:
            assert not R.user_has_item(te_ptr, te_idx, u, j)          # j not in gt_set
            assert not R.user_has_item(tr_ptr, tr_idx, u, j)          # not a train item
    flags = raw["groups"].cpu().numpy()
    ref = R.evaluate_sampled_given(users, cand, uf, itf, pop, int(tr.shape[1]), I, cred,
                                   users[flags & 1 > 0], users[flags & 2 > 0], Ks=(10, 20))
    n = users.size
    for K in (10, 20):
        for k in ("precision", "recall", "ndcg", "high_cred_recall", "low_cred_recall"):
            assert abs(res[K][k] - ref[K][k]) <= 2.0 / min(n, res[K]["high_users"] or n) + 1e-6, (K, k)
        for k in ("avg_log_popularity", "avg_self_information", "cred_utility", "item_coverage"):
            assert abs(res[K][k] - ref[K][k]) <= 1e-4 * max(abs(ref[K][k]), 1e-3) + 2.0 / n, (K, k)
        assert res[K]["high_users"] == ref[K]["high_users"] == max(round(n * 0.2), 1)
        assert res[K]["users_eval"] == n
    # deterministic for a fixed (seed, counter)
    res2 = evaluate_sampled(torch.tensor(uf, device=DEV), torch.tensor(itf, device=DEV), trc,
                            tec, I, pop, int(tr.shape[1]), cred, Ks=(10, 20))
    assert res2[20]["ndcg"] == res[20]["ndcg"] and res2[10]["item_coverage"] == res[10]["item_coverage"]


@pytest.mark.parametrize("K", [(10, 20), (3,), (1, 64)])
def test_eval_sampled_ranks_and_lists_exact_with_ties(K):
    """Integer-valued embeddings make every score an exact fp32 integer (any
    summation order), with many ties: the kernel's positive rank and top-k
    lists must be exactly the stable descending order of the candidates
    (score desc, candidate slot asc; Version-2:612-620 argsort). Pins the
    rank count's early stop for candidates outside the top k_max."""
    from bbgr.evaluation import evaluate_sampled
    U, I, d = 600, 900, 64
    tr, te = _split(U, I, 12000, 5)
    rng = np.random.default_rng(6)
    uf = rng.integers(-2, 3, size=(U, d)).astype(np.float32)
    itf = rng.integers(-2, 3, size=(I, d)).astype(np.float32)
    res = evaluate_sampled(torch.tensor(uf, device=DEV), torch.tensor(itf, device=DEV),
                           Csr(tr[0], tr[1], U, I, DEV), Csr(te[0], te[1], U, I, DEV), I,
                           np.bincount(tr[1], minlength=I), int(tr.shape[1]),
                           synthetic_credibility(U, 5), Ks=K, return_raw=True)
    raw = res.pop("_raw")
    assert raw["fails"] == 0
    users = raw["users"].cpu().numpy()
    nc = 100
    cand = raw["cand"].cpu().numpy().reshape(users.size, nc)
    pos_rank = raw["pos_rank"].cpu().numpy()
    topk = raw["topk"].cpu().numpy()
    km = max(K)
    ties = 0
    for n, u in enumerate(users):
        s = itf[cand[n]].astype(np.int64) @ uf[u].astype(np.int64)
        order = np.lexsort((np.arange(nc), -s))          # score desc, slot asc
        ties += nc - np.unique(s).size
        assert pos_rank[n] == int(np.nonzero(order == 0)[0][0]), n
        np.testing.assert_array_equal(topk[n], cand[n][order[:km]])
    assert ties > users.size * 10          # the case really is tie-heavy


def test_eval_known_ranking():
    """Hand case: one user, item scores fixed, pos guaranteed top-1."""
    from bbgr.evaluation import evaluate_sampled
    U, I, d = 1, 300, 64
    tr = np.array([[0], [1]], np.int32)
    te = np.array([[0], [0]], np.int32)
    uf = np.zeros((U, d), np.float32)
    uf[0, 0] = 1.0
    itf = np.zeros((I, d), np.float32)
    itf[:, 0] = -1.0
    itf[0, 0] = 5.0                       # the test item beats every negative
    res = evaluate_sampled(torch.tensor(uf, device=DEV), torch.tensor(itf, device=DEV),
                           Csr(tr[0], tr[1], U, I, DEV), Csr(te[0], te[1], U, I, DEV), I,
                           np.zeros(I), 1, np.ones(U), Ks=(1, 10))
    assert res[1]["recall"] == 1.0 and res[1]["precision"] == 1.0 and res[1]["ndcg"] == 1.0
    assert res[10]["precision"] == pytest.approx(0.1)


def _full_case(U, I, E, d, seed, heavy_user=False):
    tr, te = _split(U, I, E, seed)
    if heavy_user:   # user 0 has trained all but 5 items: its top-20 ends in -1e9 entries
        keep = tr[0] != 0
        tr = np.concatenate([tr[:, keep], np.stack([np.zeros(I - 5, np.int32),
                                                    np.arange(5, I, dtype=np.int32)])], axis=1)
        te = np.concatenate([te[:, te[0] != 0], np.array([[0], [1]], np.int32)], axis=1)
    rng = np.random.default_rng(seed + 1)
    uf = rng.normal(size=(U, d)).astype(np.float32)
    itf = rng.normal(size=(I, d)).astype(np.float32)
    return tr, te, uf, itf


@pytest.mark.parametrize("d,U,I,Ks", [(64, 2000, 1500, (10, 20)), (64, 700, 4099, (5, 32)),
                                      (128, 300, 777, (16,)), (64, 130, 60, (20,))])
def test_eval_full_bitexact_vs_c_oracle(d, U, I, Ks):
    """bbgr_eval_full top-K ids AND scores are bit-identical to the C oracle's
    fma chain (oracle/csrc/eval_full.c); metrics equal the reference's metric
    loop (oracle evaluate_given_topk) on those lists. Covers item splits,
    ragged user / item tiles, KM = 16/24/32, d = 128, n_items < 128."""
    from bbgr.evaluation import evaluate_full
    from oracle import native as N
    tr, te, uf, itf = _full_case(U, I, 20 * U, d, 11, heavy_user=True)
    trc, tec = Csr(tr[0], tr[1], U, I, DEV), Csr(te[0], te[1], U, I, DEV)
    pop = np.bincount(tr[1], minlength=I)
    cred = synthetic_credibility(U, 4)
    res = evaluate_full(torch.tensor(uf, device=DEV), torch.tensor(itf, device=DEV), trc, tec, I,
                        pop, int(tr.shape[1]), cred, Ks=Ks, return_raw=True)
    raw = res.pop("_raw")
    users = raw["users"].cpu().numpy()
    topk = raw["topk"].cpu().numpy()
    score = raw["topk_score"].cpu().numpy()
    tr_ptr, tr_idx = R.edges_to_user_csr(tr, U)
    te_ptr, te_idx = R.edges_to_user_csr(te, U)
    o_items, o_scores = N.full_topk(users, tr_ptr, tr_idx, uf, itf, max(Ks))
    o_items = np.where(np.isneginf(o_scores), -1, o_items)
    np.testing.assert_array_equal(topk, o_items)
    np.testing.assert_array_equal(score.view(np.uint32), o_scores.view(np.uint32))
    flags = raw["groups"].cpu().numpy()
    ref = R.evaluate_given_topk(users, o_items, te_ptr, te_idx, pop, int(tr.shape[1]), I, cred,
                                users[flags & 1 > 0], users[flags & 2 > 0], Ks=Ks)
    for K in Ks:
        for k in ref[K]:
            assert res[K][k] == pytest.approx(ref[K][k], rel=1e-9, abs=1e-12), (K, k)
        assert res[K]["mode"] == "full" and res[K]["users_eval"] == users.size


def test_eval_full_matches_reference_ranking():
    """Against the reference's own ranking expression (numpy fp32 product-sum,
    -1e9 mask, argsort): identical lists except near-ties of fp32 noise."""
    from bbgr.evaluation import evaluate_full
    U, I, d = 500, 2000, 64
    tr, te, uf, itf = _full_case(U, I, 8000, d, 21)
    trc, tec = Csr(tr[0], tr[1], U, I, DEV), Csr(te[0], te[1], U, I, DEV)
    res = evaluate_full(torch.tensor(uf, device=DEV), torch.tensor(itf, device=DEV), trc, tec, I,
                        np.bincount(tr[1], minlength=I), int(tr.shape[1]), np.ones(U), Ks=(20,),
                        return_raw=True)
    raw = res.pop("_raw")
    users = raw["users"].cpu().numpy()
    topk = raw["topk"].cpu().numpy()
    tr_ptr, tr_idx = R.edges_to_user_csr(tr, U)
    ref = R.full_ranking_reference_style(users, tr_ptr, tr_idx, uf, itf, 20)
    same = (topk == ref).all(axis=1)
    assert same.mean() >= 0.97
    s64 = uf.astype(np.float64) @ itf.T.astype(np.float64)
    for b in np.where(~same)[0]:
        u = users[b]
        a, r = np.sort(s64[u, topk[b]])[::-1], np.sort(s64[u, ref[b]])[::-1]
        np.testing.assert_allclose(a, r, rtol=1e-5, atol=1e-5)


V2_KEYS = {"precision", "recall", "ndcg", "item_coverage", "avg_log_popularity",
           "avg_self_information", "cred_utility", "high_cred_recall", "low_cred_recall",
           "high_users", "low_users", "users_eval", "mode"}


@pytest.mark.parametrize("family", ["v2_pop", "method_a", "cu_fair", "plain"])
def test_evaluate_with_the_reference_signatures(family):
    """evaluate_sampled / evaluate_full_ranking exported by each drop-in module
    with its script's signature: (model, train_csr, test_csr, num_items,
    device[, item_pop, total_train_interactions, cred_np]) with host
    (indptr, indices) CSRs from edges_to_user_csr, returning the script's
    dictionary per K (Version-2: the full set of keys; the older scripts:
    precision / recall / ndcg / users_eval / mode). The values are
    bbgr.evaluation's on the model's final tables and device CSRs built from
    the edges, bit for bit (the host-CSR conversion loses nothing)."""
    from bbgr import evaluation as EV
    from bbgr import host_sampler as HS
    from bbgr import lightgcn as SYM
    from bbgr import lightgcn_cu as CU
    from bbgr import lightgcn_cu_pop as V2
    from bbgr import lightgcn_cu_pop_long_tail_exposure as MA
    U, I, d = 600, 900, 64
    tr, te = _split(U, I, 12000, 31)
    cred = synthetic_credibility(U, 31)
    if family == "v2_pop":
        mod, m = V2, V2.LightGCN(U, I, d, 3, *V2.build_message_passing_mats(
            tr, U, I, torch.as_tensor(cred), DEV)).to(DEV)
    elif family == "method_a":
        mod, m = MA, MA.LightGCN(U, I, d, 3, *MA.build_message_passing_mats(
            tr, U, I, torch.as_tensor(cred), DEV)).to(DEV)
    elif family == "cu_fair":
        M_ui, M_iu, _ = CU.build_cred_weighted_mats(tr, U, I, cred, DEV)
        mod, m = CU, CU.CredLightGCN(U, I, d, 3, M_ui, M_iu).to(DEV)
    else:
        mod, m = SYM, SYM.LightGCN(U, I, d, 3, SYM.build_norm_adj(tr, U, I, DEV)).to(DEV)
    tr_csr, te_csr = HS.edges_to_user_csr(tr, U), HS.edges_to_user_csr(te, U)
    pop = np.bincount(tr[1].astype(np.int64), minlength=I).astype(np.float32)
    with torch.no_grad():
        ue, ie = m.final_embeddings() if family == "cu_fair" else m.get_user_item_emb()
        ue, ie = torch.as_tensor(ue).clone(), torch.as_tensor(ie).clone()
    trc, tec = Csr(tr[0], tr[1], U, I, DEV), Csr(te[0], te[1], U, I, DEV)
    v2 = family == "v2_pop"
    extra = (pop, int(tr.shape[1]), cred) if v2 else ()
    want_pop, want_total, want_cred = (pop, int(tr.shape[1]), cred) if v2 else \
        (pop, int(tr.shape[1]), np.ones(U, np.float32))
    got = mod.evaluate_sampled(m, tr_csr, te_csr, I, DEV, *extra)
    # the wrapper's host parts: the reference's users, groups, credibility mean
    # and numpy candidate stream
    users = np.where(np.diff(te_csr[0]) > 0)[0].astype(np.int64)
    flags = EV.cred_group_flags(users, want_cred, 0.2)
    cu = float(np.add.accumulate(want_cred[users].astype(np.float64))[-1]) / users.size
    cand = EV.draw_candidates(np.random.default_rng(42 + 999), users, tr_csr, te_csr, I, 99)
    host = dict(users=torch.from_numpy(users), groups=torch.from_numpy(flags), cred_utility=cu)
    want = EV.evaluate_sampled(ue, ie, trc, tec, I, want_pop, want_total, want_cred,
                               cand=cand, **host)
    checks = [(got, want, "sampled(1pos+neg)")]
    if hasattr(mod, "evaluate_full_ranking"):
        checks.append((mod.evaluate_full_ranking(m, tr_csr, te_csr, I, DEV, *extra),
                       EV.evaluate_full(ue, ie, trc, tec, I, want_pop, want_total, want_cred,
                                        **host),
                       "full"))
    for got, want, mode in checks:
        assert sorted(got) == [10, 20]
        for K in (10, 20):
            keys = V2_KEYS | ({"negatives"} if mode != "full" else set()) if v2 else \
                {"precision", "recall", "ndcg", "users_eval", "mode"} | \
                ({"negatives"} if mode != "full" else set())
            assert set(got[K]) == keys, (family, mode)
            assert got[K]["mode"] == mode
            for k in got[K]:
                assert got[K][k] == want[K][k], (family, mode, K, k)
    with pytest.raises(RuntimeError, match="No users with test interactions"):
        empty = (np.zeros(U + 1, np.int64), np.zeros(0, np.int64))
        mod.evaluate_sampled(m, tr_csr, empty, I, DEV, *extra)


@pytest.mark.parametrize("family", ["v2_pop", "method_a", "cu_fair", "plain"])
def test_reference_signature_evaluation_is_the_reference_loop(family):
    """Each drop-in module's evaluate_sampled / evaluate_full_ranking against the
    reference's whole loop restated on the CPU (Version-2/lighgcn_cu_pop.py:
    536-752; lightgcn.py:398-520, lightgcn_cu.py:488-560 and version_1 for the
    older families), on a C1-sized model (943 users x 1682 items, 100K edges,
    80/20 split) with heavily tied credibilities (0.0 / 1.0 / 0.5):
    - sampled: the restatement draws pos and negatives from
      np.random.default_rng(seed + 999) itself (numpy's integers, gt_set and
      user_has_item rejection), groups by np.argsort: the package's candidates
      equal it exactly, its Generator ends in the same state, the integer
      results (users, group sizes, coverage counts) are equal and the floats
      agree to 1e-6 relative;
    - full ranking: the restatement ranks by the kernel's score arithmetic
      (oracle/csrc/eval_full.c, one fp32 fma chain per score; the reference's
      own torch reduction order is unspecified), then runs the reference's
      metric loop with its groups: integers equal, floats to 1e-6."""
    from bbgr import evaluation as EV
    from bbgr import host_sampler as HS
    from bbgr import lightgcn as SYM
    from bbgr import lightgcn_cu as CU
    from bbgr import lightgcn_cu_pop as V2
    from bbgr import lightgcn_cu_pop_long_tail_exposure as MA
    from oracle import native as N
    U, I, d = 943, 1682, 64
    tr, te = _split(U, I, 100_000, 41)
    rng = np.random.default_rng(41)
    cred = rng.choice(np.array([0.0, 1.0, 0.5], np.float32), U, p=[0.45, 0.45, 0.1])
    torch.manual_seed(41)
    if family == "v2_pop":
        mod, m = V2, V2.LightGCN(U, I, d, 3, *V2.build_message_passing_mats(
            tr, U, I, torch.as_tensor(cred), DEV)).to(DEV)
    elif family == "method_a":
        mod, m = MA, MA.LightGCN(U, I, d, 3, *MA.build_message_passing_mats(
            tr, U, I, torch.as_tensor(cred), DEV)).to(DEV)
    elif family == "cu_fair":
        M_ui, M_iu, _ = CU.build_cred_weighted_mats(tr, U, I, cred, DEV)
        mod, m = CU, CU.CredLightGCN(U, I, d, 3, M_ui, M_iu).to(DEV)
    else:
        mod, m = SYM, SYM.LightGCN(U, I, d, 3, SYM.build_norm_adj(tr, U, I, DEV)).to(DEV)
    tr_csr, te_csr = HS.edges_to_user_csr(tr, U), HS.edges_to_user_csr(te, U)
    pop = np.bincount(tr[1].astype(np.int64), minlength=I)
    total = int(tr.shape[1])
    v2 = family == "v2_pop"
    extra = (pop, total, cred) if v2 else ()
    r_cred = cred if v2 else np.ones(U, np.float32)
    with torch.no_grad():
        ue, ie = m.final_embeddings() if family == "cu_fair" else m.get_user_item_emb()
        uf, itf = (torch.as_tensor(x).clone().cpu().numpy() for x in (ue, ie))
    users = np.where(np.diff(te_csr[0]) > 0)[0].astype(np.int64)
    hi, lo = R.make_cred_groups(users, r_cred, 0.2)
    # -- sampled
    got = EV.evaluate_sampled_reference(m, tr_csr, te_csr, I, DEV, *extra, return_raw=True)
    raw = got.pop("_raw")
    r_rng = np.random.default_rng(42 + 999)
    want, cands = R.evaluate_sampled_reference_style(*tr_csr, *te_csr, uf, itf, I, pop, total,
                                                     r_cred, Ks=(10, 20), n_neg=99, pct=0.2,
                                                     rng=r_rng)
    np.testing.assert_array_equal(raw["cand"].cpu().numpy(), np.asarray(cands))
    assert raw["rng_state"] == r_rng.bit_generator.state
    flags = raw["groups"].cpu().numpy()
    assert set(users[flags & 1 > 0].tolist()) == set(hi.tolist())
    assert set(users[flags & 2 > 0].tolist()) == set(lo.tolist())
    # the module export is the same call
    exp = mod.evaluate_sampled(m, tr_csr, te_csr, I, DEV, *extra)
    for K in (10, 20):
        assert exp[K] == got[K]
    # -- full ranking (the scripts that have it)
    checks = [(got, want)]
    if hasattr(mod, "evaluate_full_ranking"):
        fgot = mod.evaluate_full_ranking(m, tr_csr, te_csr, I, DEV, *extra)
        o_items, o_scores = N.full_topk(users, *tr_csr, uf, itf, 20)
        o_items = np.where(np.isneginf(o_scores), -1, o_items)
        fwant = R.evaluate_given_topk(users, o_items, *te_csr, pop, total, I, r_cred, hi, lo,
                                      Ks=(10, 20))
        checks.append((fgot, fwant))
    for g, w in checks:
        for K in (10, 20):
            for k, v in g[K].items():
                if k in ("mode", "negatives"):
                    continue
                if k in w[K] and isinstance(w[K][k], int):
                    assert v == w[K][k], (family, K, k)
                elif k in w[K]:
                    assert v == pytest.approx(w[K][k], rel=1e-6, abs=1e-12), (family, K, k)
            if "item_coverage" in g[K]:   # the coverage numerator is an integer
                assert round(g[K]["item_coverage"] * I) == round(w[K]["item_coverage"] * I)
            assert g[K]["users_eval"] == users.size
