"""Synthetic bipartite graphs and inputs of the BASELINE configurations.

There is no network and the reference's Amazon data is absent, so every
workload is generated here (seed = config number), SURVEY §8(d):

  * edges: unique (u, i) pairs, int32 [2, E] like train_edges.npy
    (Version-2/lighgcn_cu_pop.py:299-301). C1 draws users/items uniformly;
    C2..C5 give users a 1+Geometric degree (mean E/U) and draw items by Zipf
    rank weight (r+1)^-0.8 over a random relabelling of item ids.
  * credibility: ones (what every Version-2 log ran with) or
    Beta(1.3, 17) clipped to [0,1] with 5% of users at 1.0
    (mimics version_1/lightgcn_cu_fair.out:15-16).
  * embeddings: xavier_uniform_ like Version-2/lighgcn_cu_pop.py:469-470.
"""
from __future__ import annotations

import numpy as np

CONFIGS = {
    "C1": dict(num_users=943, num_items=1682, num_edges=100_000, emb_dim=64, num_layers=3,
               batch=4096, items="uniform"),
    "C2": dict(num_users=100_000, num_items=50_000, num_edges=1_000_000, emb_dim=64,
               num_layers=3, batch=4096, items="zipf"),
    "C3": dict(num_users=5_000_000, num_items=1_000_000, num_edges=50_000_000, emb_dim=128,
               num_layers=3, batch=8192, items="zipf"),
    "C4": dict(num_users=5_000_000, num_items=1_000_000, num_edges=50_000_000, emb_dim=64,
               num_layers=3, batch=8192, items="zipf"),
    "C5": dict(num_users=10_000_000, num_items=2_000_000, num_edges=500_000_000, emb_dim=256,
               num_layers=4, batch=8192, items="zipf"),
}
CONFIG_SEED = {"C1": 1, "C2": 2, "C3": 3, "C4": 4, "C5": 5}


def _zipf_sampler(num_items: int, s: float, rng: np.random.Generator, item_seed: int):
    w = np.power(np.arange(1, num_items + 1, dtype=np.float64), -s)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    # popularity rank -> item id relabelling: its own stream, so shards drawn
    # with different seeds but one item_seed agree on which items are popular
    relabel = np.random.default_rng([item_seed, 0xA11CE]).permutation(num_items).astype(np.int64)

    def draw(n: int) -> np.ndarray:
        r = np.searchsorted(cdf, rng.random(n), side="right")
        np.minimum(r, num_items - 1, out=r)
        return relabel[r]

    return draw


def synthetic_edges(num_users: int, num_items: int, num_edges: int, seed: int,
                    items: str = "zipf", zipf_s: float = 0.8,
                    duplicates: int = 0, item_seed: int | None = None) -> np.ndarray:
    """int32 [2, E] unique (u, i) pairs (+ `duplicates` repeated pairs appended,
    for the coalesce-equivalence parity cases). `item_seed` (default: seed) fixes
    the item popularity order independently of the edge draws."""
    rng = np.random.default_rng(seed)
    U, I, E = int(num_users), int(num_items), int(num_edges)
    if E > U * I:
        raise ValueError("more edges than user-item pairs")
    if items == "uniform":
        keys = np.unique(rng.integers(0, U * I, size=int(E * 1.1) + 16, dtype=np.int64))
        while keys.size < E:
            keys = np.unique(np.concatenate(
                [keys, rng.integers(0, U * I, size=E - keys.size + 16, dtype=np.int64)]))
        keys = rng.permutation(keys)[:E]
    else:
        mean = E / U
        deg = rng.geometric(min(1.0, 1.0 / mean), size=U).astype(np.int64)
        np.minimum(deg, I, out=deg)
        diff = E - int(deg.sum())
        while diff != 0:   # nudge random users until the degrees sum to E
            pick = rng.integers(0, U, size=abs(diff))
            if diff > 0:
                np.add.at(deg, pick, 1)
                np.minimum(deg, I, out=deg)
            else:
                np.subtract.at(deg, pick, 1)
                np.maximum(deg, 1 if E >= U else 0, out=deg)
            diff = E - int(deg.sum())
        draw = _zipf_sampler(I, zipf_s, rng, seed if item_seed is None else item_seed)
        users = np.repeat(np.arange(U, dtype=np.int64), deg)
        keys = users * I + draw(E)
        keys.sort()
        dup = np.zeros(E, dtype=bool)
        dup[1:] = keys[1:] == keys[:-1]
        uniq = keys[~dup]
        pending_users = keys[dup] // I
        accepted = []
        acc_set = np.empty(0, dtype=np.int64)
        while pending_users.size:
            cand = pending_users * I + draw(pending_users.size)
            cu, first = np.unique(cand, return_index=True)
            ok = np.zeros(cand.size, dtype=bool)
            ok[first] = True
            pos = np.searchsorted(uniq, cand)
            pos = np.minimum(pos, uniq.size - 1)
            ok &= uniq[pos] != cand
            ok &= ~np.isin(cand, acc_set)
            accepted.append(cand[ok])
            acc_set = np.concatenate([acc_set, cand[ok]])
            pending_users = pending_users[~ok]
        keys = np.concatenate([uniq] + accepted)
        keys = keys[rng.permutation(keys.size)]
    edges = np.empty((2, E + duplicates), dtype=np.int32)
    edges[0, :E] = keys // I
    edges[1, :E] = keys % I
    if duplicates:
        j = rng.integers(0, E, size=duplicates)
        edges[:, E:] = edges[:, j]
    return edges


def config_edges(name: str, duplicates: int = 0) -> np.ndarray:
    c = CONFIGS[name]
    return synthetic_edges(c["num_users"], c["num_items"], c["num_edges"], CONFIG_SEED[name],
                           items=c["items"], duplicates=duplicates)


def shard_edges_weak(name: str, rank: int) -> np.ndarray:
    """Weak scaling: rank r owns a full config-sized user shard (its own users,
    local ids) over the SAME item set and item popularity; rank 0's shard is
    exactly config_edges(name)."""
    c = CONFIGS[name]
    return synthetic_edges(c["num_users"], c["num_items"], c["num_edges"],
                           CONFIG_SEED[name] + 7919 * rank, items=c["items"],
                           item_seed=CONFIG_SEED[name])


def user_ranges(num_users: int, world: int) -> np.ndarray:
    """Contiguous user ranges of (almost) equal size: bounds[world + 1]."""
    return np.array([num_users * g // world for g in range(world + 1)], dtype=np.int64)


def shard_edges_strong(name: str, rank: int, world: int) -> tuple[np.ndarray, int, int]:
    """Strong scaling of a graph too large to draw on every rank (C5: 500M
    edges): rank r draws only ITS users' edges — user range r of
    user_ranges(U, world), edges in proportion, same degree law, same item
    popularity order — so the union over ranks is one config-sized graph.
    Returns (local edges int32 [2, E_r] with local user ids, lo, hi)."""
    c = CONFIGS[name]
    b = user_ranges(c["num_users"], world)
    lo, hi = int(b[rank]), int(b[rank + 1])
    e_lo = c["num_edges"] * lo // c["num_users"]
    e_hi = c["num_edges"] * hi // c["num_users"]
    e = synthetic_edges(hi - lo, c["num_items"], e_hi - e_lo,
                        CONFIG_SEED[name] + 7919 * rank + 104729 * world,
                        items=c["items"], item_seed=CONFIG_SEED[name])
    return e, lo, hi


def synthetic_credibility(num_users: int, seed: int, kind: str = "beta") -> np.ndarray:
    if kind == "ones":
        return np.ones(num_users, dtype=np.float32)
    rng = np.random.default_rng(seed + 1000)
    c = np.clip(rng.beta(1.3, 17.0, size=num_users), 0.0, 1.0)
    c[rng.random(num_users) < 0.05] = 1.0
    return c.astype(np.float32)


def xavier_tables(num_users: int, num_items: int, d: int, seed: int = 42):
    """u0 [U,d], i0 [I,d] fp32 with the xavier_uniform_ bound of each table."""
    rng = np.random.default_rng(seed)
    au, ai = np.sqrt(6.0 / (num_users + d)), np.sqrt(6.0 / (num_items + d))
    u0 = rng.uniform(-au, au, size=(num_users, d)).astype(np.float32)
    i0 = rng.uniform(-ai, ai, size=(num_items, d)).astype(np.float32)
    return u0, i0
