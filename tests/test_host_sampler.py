"""bbgr.host_sampler: the reference's host CSR helpers and samplers
(Version-2/lighgcn_cu_pop.py:309-376, the loop :835-849; lightgcn.py:296-303)
reproduced bit for bit — identical samples AND an identical numpy Generator
state afterwards — against the oracle's literal restatement
(oracle/ref_numpy.py, which calls rng.choice(p=) per popularity draw as the
reference does) and against the committed C4 first-batch fixture
(tests/golden/make_golden_sampler.py)."""
import json
import os
import time

import numpy as np
import pytest

import bbgr  # noqa: F401
from bbgr import host_sampler as H
from oracle import ref_numpy as R

HERE = os.path.dirname(os.path.abspath(__file__))


def _graph(U, I, E, seed, dup=0, full_users=(), deg1_users=()):
    rng = np.random.default_rng(seed)
    u = rng.integers(0, U, E)
    it = rng.integers(0, I, E)
    if dup:
        u = np.concatenate([u, u[:dup]])
        it = np.concatenate([it, it[:dup]])
    for fu in full_users:   # a user who has every item: pop draws all rejected
        u = np.concatenate([u, np.full(I, fu)])
        it = np.concatenate([it, np.arange(I)])
    keep = ~np.isin(u, np.asarray(deg1_users, dtype=np.int64))
    u, it = u[keep], it[keep]
    for k, du in enumerate(deg1_users):   # one edge: integers(s, s + 1) draws nothing
        u = np.concatenate([u, [du]])
        it = np.concatenate([it, [k % I]])
    return np.stack([u, it]).astype(np.int32)


def _literal_csr(edges, U):
    """Version-2/lighgcn_cu_pop.py:309-327 as written (mergesort by user, then
    np.sort per row in a Python loop)."""
    u = edges[0].astype(np.int64)
    it = edges[1].astype(np.int64)
    order = np.argsort(u, kind="mergesort")
    u, it = u[order], it[order]
    counts = np.bincount(u, minlength=U)
    indptr = np.zeros(U + 1, dtype=np.int64)
    indptr[1:] = np.cumsum(counts)
    indices = it.copy()
    for user in range(U):
        s, e = indptr[user], indptr[user + 1]
        if e - s > 1:
            indices[s:e] = np.sort(indices[s:e])
    return indptr, indices


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_edges_to_user_csr_is_the_reference_loop(seed):
    U, I = 300, 200
    e = _graph(U, I, 4000, seed, dup=50)
    ip, ix = H.edges_to_user_csr(e, U)
    lp, lx = _literal_csr(e, U)
    assert ip.dtype == np.int64 and ix.dtype == np.int64
    np.testing.assert_array_equal(ip, lp)
    np.testing.assert_array_equal(ix, lx)
    # empty edge list and users past the last edge
    ip0, ix0 = H.edges_to_user_csr(np.zeros((2, 0), np.int32), 5)
    assert ip0.tolist() == [0] * 6 and ix0.size == 0


def test_user_has_item_and_pos_match_the_oracle():
    U, I = 200, 150
    e = _graph(U, I, 3000, 5, deg1_users=(3, 4))
    ip, ix = H.edges_to_user_csr(e, U)
    for u in range(U):
        for i in range(0, I, 7):
            assert H.user_has_item(ip, ix, u, i) == R.user_has_item(ip, ix, u, i)
    a, b = np.random.default_rng(11), np.random.default_rng(11)
    for u in range(U):
        assert H.sample_pos_item(ip, ix, u, a) == R.sample_pos_item(ip, ix, u, b)
    assert a.bit_generator.state == b.bit_generator.state


@pytest.mark.parametrize("seed", [0, 7, 42])
def test_neg_samplers_match_the_oracle_draw_for_draw(seed):
    U, I = 120, 90
    # user 0 holds every item (max_tries exhausted -> the uniform loop, which
    # also rejects forever: that user is only asked for a positive), users 5, 6
    # a single edge
    e = _graph(U, I, 2500, seed, full_users=(1,), deg1_users=(5, 6))
    ip, ix = H.edges_to_user_csr(e, U)
    pp = R.pop_prob(e, I)
    a, b = np.random.default_rng(seed), np.random.default_rng(seed)
    for u in range(2, U):
        got = H.sample_neg_item_popmix(ip, ix, u, I, a, pp, 0.7, 50)
        want = R.sample_neg_item_popmix(ip, ix, u, I, b, pp, 0.7, 50)
        assert got == want, u
        assert H.sample_neg_item(ip, ix, u, I, a) == R.sample_neg_item(ip, ix, u, I, b)
    assert a.bit_generator.state == b.bit_generator.state


def test_max_tries_exhausted_falls_back_to_uniform_like_the_reference():
    """A user holding all but one item: pop draws are rejected until max_tries
    runs out (small max_tries), then the uniform loop finds the free item."""
    I = 40
    u = np.zeros(I - 1, np.int64)
    it = np.arange(1, I)
    e = np.stack([u, it]).astype(np.int32)
    ip, ix = H.edges_to_user_csr(e, 1)
    pp = R.pop_prob(e, I)
    for seed in range(5):
        a, b = np.random.default_rng(seed), np.random.default_rng(seed)
        assert H.sample_neg_item_popmix(ip, ix, 0, I, a, pp, 0.9, 3) == 0
        assert R.sample_neg_item_popmix(ip, ix, 0, I, b, pp, 0.9, 3) == 0
        assert a.bit_generator.state == b.bit_generator.state


@pytest.mark.parametrize("popmix", [True, False])
def test_batch_loop_matches_the_reference_loop(popmix):
    U, I = 400, 300
    e = _graph(U, I, 6000, 3, dup=30, deg1_users=(9,))
    ip, ix = H.edges_to_user_csr(e, U)
    pp = R.pop_prob(e, I)
    users = np.random.default_rng(1).permutation(U + 0)   # includes users with no edges
    a, b = np.random.default_rng(42), np.random.default_rng(42)
    if popmix:
        got = H.sample_batch(ip, ix, users, I, a, pp, 0.7, 50)
        want = R.sample_batch_reference_style(ip, ix, users, I, b, pp, 0.7, 50)
    else:
        got = H.sample_batch(ip, ix, users, I, a)
        want = R.sample_batch_uniform_reference_style(ip, ix, users, I, b)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)
    assert a.bit_generator.state == b.bit_generator.state


def test_invalid_pop_prob_raises_like_numpy_choice():
    rng = np.random.default_rng(0)
    ip, ix = H.edges_to_user_csr(np.array([[0], [0]], np.int32), 1)
    for bad in (np.array([0.5, 0.6, -0.1]), np.array([0.2, 0.2, 0.2]), np.array([0.5, 0.5])):
        with pytest.raises(ValueError):
            rng.choice(3, p=bad)
        with pytest.raises(ValueError):
            H.sample_neg_item_popmix(ip, ix, 0, 3, np.random.default_rng(0), bad, 1.0, 5)


def test_cached_cdf_follows_a_new_array_and_an_in_place_change():
    p1 = np.full(8, 1 / 8)
    c1 = H.pop_cdf(p1, 8).copy()
    p1[:4], p1[4:] = 0.2, 0.05
    c2 = H.pop_cdf(p1, 8)
    want = p1.cumsum()
    want /= want[-1]
    assert not np.array_equal(c1, c2) and np.array_equal(c2, want)


def test_c4_first_batch_is_the_reference_loop_bit_for_bit():
    """The first training batch of a seeded Version-2 run on the C4 graph
    (U=5M, I=1M, E=50M, B=8192, pop-mix 0.7 / gamma 0.75 / 50 tries): users,
    positives, negatives and the Generator's final state equal the fixture the
    reference-style loop wrote (rng.choice(p=) over 1M items per popularity
    draw: ~1 min of host time, tests/golden/make_golden_sampler.py), and the
    batch takes well under a second here (the reference loop: 24.8 s on the
    GPU box's host, BENCH_r04)."""
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_golden_sampler import c4_first_batch_inputs
    g = np.load(os.path.join(HERE, "golden", "sampler_c4_b8192.npz"))
    indptr, indices, users, I, pp, rng, e = c4_first_batch_inputs(with_edges=True)
    ip, ix = H.edges_to_user_csr(e, indptr.size - 1)   # the package's CSR == the oracle's
    del e
    np.testing.assert_array_equal(ip, indptr)
    np.testing.assert_array_equal(ix, indices)
    del ip, ix
    np.testing.assert_array_equal(users, g["batch_users"])
    H.pop_cdf(pp, I)   # the one-time CDF (a training run builds it once)
    t0 = time.perf_counter()
    used, pos, neg = H.sample_batch(indptr, indices, users, I, rng, pp, 0.7, 50)
    dt = time.perf_counter() - t0
    np.testing.assert_array_equal(used, g["used"])
    np.testing.assert_array_equal(pos, g["pos"])
    np.testing.assert_array_equal(neg, g["neg"])
    assert rng.bit_generator.state == json.loads(str(g["state"]))
    assert dt < 1.0, f"C4 batch took {dt:.2f} s"
