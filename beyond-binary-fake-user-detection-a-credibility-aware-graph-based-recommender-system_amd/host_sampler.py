"""The reference's host-side CSR helpers and samplers, bit-exact and fast.

Same names, signatures, return values and numpy random stream as
Version-2/lighgcn_cu_pop.py:309-376 (and lightgcn.py:259-303 /
lightgcn_cu.py:259-302 for the uniform negative sampler):

  edges_to_user_csr(edges_2xE, num_users) -> (indptr int64, indices int64)   :309-327
  user_has_item(indptr, indices, user, item) -> bool                         :330-336
  sample_pos_item(indptr, indices, user, rng) -> int | None                  :339-343
  sample_neg_item_popmix(indptr, indices, user, num_items, rng, pop_prob,
                         mix_pop, max_tries) -> int                          :349-376
  sample_neg_item(indptr, indices, user, num_items, rng) -> int   lightgcn.py:296-303
  sample_batch(indptr, indices, batch_users, num_items, rng, pop_prob=None,
               mix_pop=0.7, max_tries=50) -> (users, pos, neg)   the loop :835-849

For a caller that needs the reference's exact training batches (a seeded run
reproduced draw for draw) rather than the device sampler's Philox stream
(bbgr.sampler). The one costly call of the reference loop is
`rng.choice(num_items, p=pop_prob)`: numpy validates p, forms
`cdf = p.cumsum(); cdf /= cdf[-1]` and draws ONE `random()` searched with
`cdf.searchsorted(u, side="right")` — O(I) per draw (1M items at C4: the
loop's 24.8 s for a B = 8192 batch, BENCH_r04 cpu_baseline.components_s).
Here the normalised CDF is built once per pop_prob array (the same numpy
operations, so the same doubles) and each draw is the same single
`rng.random()` and the same search: O(log I), and the Generator consumes
exactly the bits it would (identical samples and identical
`rng.bit_generator.state` afterwards, tests/test_host_sampler.py). Every
other draw (`rng.random()`, `rng.integers(...)`) is the reference's own call
with the same arguments, so bounded-integer buffering and the no-draw case
`integers(s, s + 1)` behave exactly as there.

numpy's argument checks of choice(p=) run once per pop_prob array (same
errors: ValueError for a negative, unnormalised or wrongly sized p); an
array changed in place after its first use must be passed as a new array
(its cached CDF is keyed by identity, checked by a 1024-entry fingerprint).
"""
from __future__ import annotations

import weakref

import numpy as np

__all__ = ["edges_to_user_csr", "user_has_item", "sample_pos_item", "sample_neg_item",
           "sample_neg_item_popmix", "sample_batch", "pop_cdf"]


def edges_to_user_csr(edges_2xE: np.ndarray, num_users: int):
    """Version-2/lighgcn_cu_pop.py:309-327: rows by user (mergesort, stable),
    then each row's items sorted ascending; duplicate pairs kept. One radix-
    friendly sort of the composite key (user, item) gives exactly those rows:
    inside a row equal keys are equal items, so stability is moot."""
    u = np.asarray(edges_2xE[0]).astype(np.int64)
    it = np.asarray(edges_2xE[1]).astype(np.int64)
    counts = np.bincount(u, minlength=num_users)
    indptr = np.zeros(num_users + 1, dtype=np.int64)
    indptr[1:] = np.cumsum(counts)
    if it.size == 0:
        return indptr, it.copy()
    lo = int(it.min())
    span = int(it.max()) - lo + 1
    keys = u * span + (it - lo)
    keys.sort()
    return indptr, keys % span + lo


def user_has_item(indptr, indices, user: int, item: int) -> bool:
    """Version-2/lighgcn_cu_pop.py:330-336 (binary search in the sorted row)."""
    start, end = indptr[user], indptr[user + 1]
    if start == end:
        return False
    arr = indices[start:end]
    j = arr.searchsorted(item)
    return bool(j < (end - start) and arr[j] == item)


def sample_pos_item(indptr, indices, user: int, rng: np.random.Generator):
    """Version-2/lighgcn_cu_pop.py:339-343."""
    start, end = indptr[user], indptr[user + 1]
    if start == end:
        return None
    return int(indices[rng.integers(start, end)])


def sample_neg_item(indptr, indices, user: int, num_items: int, rng: np.random.Generator):
    """lightgcn.py:296-303 / lightgcn_cu.py:295-302: uniform, rejected while
    the user has the item."""
    while True:
        j = int(rng.integers(0, num_items))
        if not user_has_item(indptr, indices, user, j):
            return j


class _Cdf:
    __slots__ = ("cdf", "n", "fp", "ref", "__weakref__")


_CACHE: dict = {}
_FP_POINTS = 1024


def _fingerprint(p: np.ndarray) -> bytes:
    step = max(1, p.size // _FP_POINTS)
    return p[::step].tobytes() + p[-1:].tobytes()


def pop_cdf(pop_prob: np.ndarray, num_items: int) -> np.ndarray:
    """The normalised CDF numpy's Generator.choice(num_items, p=pop_prob)
    searches, with choice's argument checks, cached per pop_prob array."""
    key = id(pop_prob)
    c = _CACHE.get(key)
    if c is not None and c.ref() is pop_prob and c.n == num_items and \
            c.fp == _fingerprint(np.asarray(pop_prob)):
        return c.cdf
    n = int(num_items)
    if n <= 0:
        raise ValueError("a must be a positive integer unless no samples are taken")
    p = np.ascontiguousarray(pop_prob, dtype=np.float64)
    if p.ndim != 1:
        raise ValueError("p must be 1-dimensional")
    if p.size != n:
        raise ValueError("a and p must have same size")
    if np.logical_or.reduce(p < 0):
        raise ValueError("probabilities are not non-negative")
    atol = max(np.sqrt(np.finfo(np.float64).eps),
               np.sqrt(np.finfo(pop_prob.dtype).eps)
               if isinstance(pop_prob, np.ndarray) and np.issubdtype(pop_prob.dtype, np.floating)
               else 0.0)
    s = float(np.sum(p))   # numpy uses a Kahan sum; |s - 1| <= atol either way for valid p
    if np.isnan(s):
        raise ValueError("probabilities contain NaN")
    if abs(s - 1.0) > atol:
        raise ValueError("probabilities do not sum to 1")
    cdf = p.cumsum()
    cdf /= cdf[-1]
    c = _Cdf()
    c.cdf, c.n, c.fp = cdf, n, _fingerprint(np.asarray(pop_prob))
    try:
        c.ref = weakref.ref(pop_prob, lambda _r, k=key: _CACHE.pop(k, None))
    except TypeError:             # not weak-referenceable (a list): keep it alive
        c.ref = (lambda obj=pop_prob: obj)
    _CACHE[key] = c
    return cdf


def sample_neg_item_popmix(indptr, indices, user: int, num_items: int,
                           rng: np.random.Generator, pop_prob: np.ndarray,
                           mix_pop: float, max_tries: int):
    """Version-2/lighgcn_cu_pop.py:349-376: up to max_tries draws, each from
    pop_prob with probability mix_pop (rng.choice(p=), here one rng.random()
    searched in the cached CDF) else uniform, rejected while the user has the
    item; then uniform draws until a non-positive is found."""
    cdf = pop_cdf(pop_prob, num_items)
    for _ in range(max_tries):
        if rng.random() < mix_pop:
            j = int(cdf.searchsorted(rng.random(), side="right"))
        else:
            j = int(rng.integers(0, num_items))
        if not user_has_item(indptr, indices, user, j):
            return j
    while True:
        j = int(rng.integers(0, num_items))
        if not user_has_item(indptr, indices, user, j):
            return j


def sample_batch(indptr, indices, batch_users, num_items: int, rng: np.random.Generator,
                 pop_prob: np.ndarray | None = None, mix_pop: float = 0.7, max_tries: int = 50):
    """The per-user loop of Version-2/lighgcn_cu_pop.py:835-849 (pop_prob
    given) or lightgcn.py / lightgcn_cu.py's (pop_prob None: uniform
    negatives): (used_users, pos_items, neg_items) as int64 arrays, users with
    an empty row skipped. The same draws in the same order as calling the
    functions above per user; the loop body is inlined (bound methods, no
    per-call lookups) and the membership test searches the row slice once."""
    cdf = pop_cdf(pop_prob, num_items) if pop_prob is not None else None
    rand, ints = rng.random, rng.integers
    search = cdf.searchsorted if cdf is not None else None
    used, pos, neg = [], [], []
    for u in batch_users:
        u = int(u)
        s, e = indptr[u], indptr[u + 1]
        if s == e:
            continue
        p = int(indices[ints(s, e)])
        row = indices[s:e]
        n_row = e - s
        j = -1
        if cdf is not None:
            for _ in range(max_tries):
                if rand() < mix_pop:
                    c = int(search(rand(), side="right"))
                else:
                    c = int(ints(0, num_items))
                k = row.searchsorted(c)
                if not (k < n_row and row[k] == c):
                    j = c
                    break
        while j < 0:
            c = int(ints(0, num_items))
            k = row.searchsorted(c)
            if not (k < n_row and row[k] == c):
                j = c
        used.append(u)
        pos.append(p)
        neg.append(j)
    return (np.array(used, dtype=np.int64), np.array(pos, dtype=np.int64),
            np.array(neg, dtype=np.int64))
