"""GPU: sampled evaluation (bbgr_eval_sampled) vs the oracle restatement of
Version-2/lighgcn_cu_pop.py:536-650 on the SAME candidates.

The candidates come from the device Philox stream (numpy's PCG64 stream is not
reproduced: distributional parity), so the test (1) checks every candidate
invariant exactly and (2) feeds the device's candidates to the float64 oracle
and compares the metrics. fp32 vs float64 scores can swap a near-tie, so
per-user hit metrics may differ for at most 2 users."""
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
