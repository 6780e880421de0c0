"""CPU: the reference's sampled-evaluation candidate stream, bit for bit.

evaluate_sampled (Version-2/lighgcn_cu_pop.py:554-589; the same loop in
lightgcn.py:406-429, lightgcn_cu.py:496-519 and
version_1/lightgcn_cu_pop_long_tail_exposure.py:494-517) draws each evaluated
user's positive and negatives from np.random.default_rng(seed + 999) with
scalar Generator.integers calls and rejection. bbgr_eval_draw_candidates (host
C in libbbgr.so, no GPU) restates numpy's PCG64 and its bounded-integer path;
it must give the literal loop's candidates (oracle/ref_numpy.py, which calls
numpy itself) AND leave the Generator in numpy's own end state. The credibility
groups are the reference's np.argsort split, ties included.
"""
import numpy as np
import pytest

from bbgr import evaluation as EV
from bbgr._lib import BbgrError
from oracle import ref_numpy as R


def _csrs(U, I, E, seed, sort_train=True):
    rng = np.random.default_rng(seed)
    u = rng.integers(0, U, E)
    i = (rng.zipf(1.3, E) - 1) % I
    test = rng.random(E) < 0.2
    tr = np.stack([u[~test], i[~test]])
    te = np.stack([u[test], i[test]])
    tr_csr = R.edges_to_user_csr(tr, U)
    te_csr = R.edges_to_user_csr(te, U)
    if not sort_train:   # rows in arrival order: user_has_item's searchsorted on an unsorted row
        order = np.argsort(tr[0], kind="stable")
        tr_csr = (tr_csr[0], tr[1][order].astype(np.int64))
        te_order = np.argsort(te[0], kind="stable")
        te_csr = (te_csr[0], te[1][te_order].astype(np.int64))
    return tr_csr, te_csr


def _users(te_csr):
    return np.where(np.diff(te_csr[0]) > 0)[0].astype(np.int64)


def _check(rng_a, rng_b, users, tr_csr, te_csr, I, n_neg):
    want = R.sampled_candidates_reference_style(rng_a, users, *tr_csr, *te_csr, I, n_neg)
    got = EV.draw_candidates(rng_b, users, tr_csr, te_csr, I, n_neg)
    np.testing.assert_array_equal(got, want)
    assert rng_b.bit_generator.state == rng_a.bit_generator.state
    # the two Generators continue identically
    assert rng_a.integers(0, 1 << 40, 8).tolist() == rng_b.integers(0, 1 << 40, 8).tolist()
    return got


@pytest.mark.parametrize("seed", [42 + 999, 0, 7])
def test_candidates_and_generator_state_equal_the_reference_loop(seed):
    tr_csr, te_csr = _csrs(943, 1682, 100_000, seed % 97)
    users = _users(te_csr)
    got = _check(np.random.default_rng(seed), np.random.default_rng(seed), users, tr_csr,
                 te_csr, 1682, 99)
    assert got.shape == (users.size, 100)


def test_buffered_half_output_and_unsorted_rows():
    """A Generator holding a buffered 32-bit half (an odd number of 32-bit
    draws before), rows in arrival order (searchsorted on an unsorted train row,
    duplicate test items), small n_neg."""
    tr_csr, te_csr = _csrs(300, 500, 20_000, 3, sort_train=False)
    users = _users(te_csr)
    a, b = np.random.default_rng(5), np.random.default_rng(5)
    for g in (a, b):
        g.integers(0, 7)          # one 32-bit draw: the high half stays buffered
        assert g.bit_generator.state["has_uint32"] == 1
    _check(a, b, users, tr_csr, te_csr, 500, 5)


def test_lemire_rejections_at_a_wide_item_range():
    """n_items = 1.5 * 2^30: a quarter of the 32-bit draws fall below Lemire's
    threshold and are redrawn; the positive draw of a long test row too."""
    I = 3 << 29
    rng = np.random.default_rng(11)
    U = 50
    te = np.stack([rng.integers(0, U, 400), rng.integers(0, I, 400)])
    tr = np.stack([rng.integers(0, U, 400), rng.integers(0, I, 400)])
    tr_csr, te_csr = R.edges_to_user_csr(tr, U), R.edges_to_user_csr(te, U)
    _check(np.random.default_rng(2), np.random.default_rng(2), _users(te_csr), tr_csr, te_csr,
           I, 40)


def test_heavy_rejection_and_single_item_test_rows():
    """A user holding every item but two (most draws rejected), users with one
    test item (integers(0, 1) draws nothing), n_neg = 0."""
    I = 64
    tr = [(0, j) for j in range(I) if j not in (5, 40)] + [(1, 3), (2, 9)]
    te = [(0, 5), (1, 4), (1, 4), (2, 1), (2, 2), (2, 63)]
    tr_csr = R.edges_to_user_csr(np.array(tr).T, 3)
    te_csr = R.edges_to_user_csr(np.array(te).T, 3)
    users = _users(te_csr)
    got = _check(np.random.default_rng(1), np.random.default_rng(1), users, tr_csr, te_csr, I, 99)
    assert set(got[0, 1:].tolist()) == {40}
    _check(np.random.default_rng(1), np.random.default_rng(1), users, tr_csr, te_csr, I, 0)


def test_no_admissible_negative_raises_instead_of_looping():
    I = 4
    tr_csr = R.edges_to_user_csr(np.array([[0, 0, 0], [0, 1, 2]]), 1)
    te_csr = R.edges_to_user_csr(np.array([[0], [3]]), 1)
    with pytest.raises(BbgrError, match="no admissible negative"):
        EV.draw_candidates(np.random.default_rng(0), _users(te_csr), tr_csr, te_csr, I, 3)


def test_cred_groups_are_the_reference_argsort_split_with_ties():
    """make_cred_groups (Version-2:408-426) with many tied credibilities: the
    package's split (np.argsort, the reference's call) equals the oracle's
    restatement user for user; a stable sort would split the ties otherwise."""
    rng = np.random.default_rng(3)
    U = 5000
    cred = rng.choice(np.array([0.0, 1.0, 0.5, 0.25], np.float32), U, p=[0.4, 0.4, 0.1, 0.1])
    cred[rng.random(U) < 0.05] = np.float32(0.7)
    users = np.sort(rng.choice(U, 3000, replace=False)).astype(np.int64)
    for pct in (0.2, 0.1, 0.5, 1e-6):
        hi, lo = R.make_cred_groups(users, cred, pct)
        flags = EV.cred_group_flags(users, cred, pct)
        assert set(users[flags & 1 > 0].tolist()) == set(hi.tolist())
        assert set(users[flags & 2 > 0].tolist()) == set(lo.tolist())
        h2, l2 = EV.make_cred_groups(users, cred, pct)
        np.testing.assert_array_equal(h2, hi)
        np.testing.assert_array_equal(l2, lo)
