"""CPU, world size 2 over gloo: the shard plan and the exchange schedule of
bbgr.distributed (user-row sharding, item partial sums all-reduced per layer).

The HIP kernels cannot run here, so each rank evaluates its local products
with the float64 oracle; the partition, the edge sharding, the global item
degree all-reduce and the per-layer partial-sum all-reduce are the product's
own functions / schedule and must reproduce the unsharded propagation."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _spawn(fn, world, out):
    """mp.spawn over a rendezvous store this process holds (tests/_ports.py)."""
    from _ports import host_store
    store, port = host_store(world)
    mp.spawn(fn, args=(world, port, out), nprocs=world, join=True)
    del store


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    import bbgr  # noqa: F401
    from bbgr.distributed import global_item_indptr, partition_users, shard_edges
    from oracle import ref_numpy as R
    sys.path.insert(0, HERE)
    from _ports import init_worker
    init_worker(rank, world, port)
    g = np.load(os.path.join(HERE, "golden", "golden_small.npz"))
    U, I, E, DUP, D, K, B = (int(x) for x in g["meta"])
    e, cred, u0, i0 = g["edges"], g["cred"], g["u0"], g["i0"]
    bounds = partition_users(np.bincount(e[0], minlength=U), world)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    loc = shard_edges(e, lo, hi)
    # global item degrees by all-reduce (product code) == bincount over all edges
    deg_local = torch.as_tensor(np.bincount(loc[1], minlength=I).astype(np.int32))
    indptr_i = global_item_indptr(deg_local)
    deg_i = np.diff(indptr_i.numpy()).astype(np.float32)
    assert (deg_i == np.bincount(e[1], minlength=I)).all()
    # local factored operators with GLOBAL item scales
    deg_u = np.bincount(loc[0], minlength=hi - lo).astype(np.float32)
    a = 1.0 / np.sqrt(np.maximum(deg_u, 1.0))
    b = 1.0 / np.sqrt(np.maximum(deg_i, 1.0))
    c = cred[lo:hi]
    A_iu = R.csr64(loc[1], loc[0], np.ones(loc.shape[1]), (I, hi - lo))
    A_ui = A_iu.T.tocsr()
    u, it = u0[lo:hi].astype(np.float64), i0.astype(np.float64)
    us, is_ = [u], [it]
    for _ in range(K):   # GS schedule: partial item sums -> all-reduce -> epilogue
        t = torch.as_tensor(A_iu @ ((c * a)[:, None] * u))
        dist.all_reduce(t)
        it = b[:, None] * t.numpy()
        u = a[:, None] * (A_ui @ (b[:, None] * it))
        us.append(u)
        is_.append(it)
    np.savez(os.path.join(out, f"r{rank}.npz"), lo=lo, hi=hi, uf=np.mean(us, 0),
             itf=np.mean(is_, 0))
    dist.destroy_process_group()


def test_two_rank_schedule_matches_unsharded(tmp_path):
    from oracle import ref_numpy as R
    _spawn(_worker, 2, str(tmp_path))
    r = [np.load(tmp_path / f"r{k}.npz") for k in range(2)]
    g = np.load(os.path.join(HERE, "golden", "golden_small.npz"))
    U, I, E, DUP, D, K, B = (int(x) for x in g["meta"])
    M_ui, M_iu = R.gs_mats(g["edges"], U, I, g["cred"])
    uf, itf, _, _ = R.propagate_gs(M_ui, M_iu, g["u0"], g["i0"], K)
    assert int(r[0]["lo"]) == 0 and int(r[0]["hi"]) == int(r[1]["lo"]) and int(r[1]["hi"]) == U
    got_u = np.concatenate([r[0]["uf"], r[1]["uf"]])
    assert np.linalg.norm(got_u - uf) <= 1e-6 * np.linalg.norm(uf)
    for k in range(2):   # replicated item tables agree with the unsharded truth
        assert np.linalg.norm(r[k]["itf"] - itf) <= 1e-6 * np.linalg.norm(itf)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_partition_is_contiguous_and_edge_balanced(world):
    from bbgr.distributed import partition_users, shard_edges
    from bbgr.synthetic import synthetic_edges
    e = synthetic_edges(5000, 800, 60000, 3, items="zipf")
    deg = np.bincount(e[0], minlength=5000)
    b = partition_users(deg, world)
    assert b[0] == 0 and b[-1] == 5000 and (np.diff(b) >= 0).all()
    loads = [deg[b[g]:b[g + 1]].sum() for g in range(world)]
    assert sum(loads) == e.shape[1]
    assert max(loads) - min(loads) <= 2 * deg.max()
    parts = [shard_edges(e, b[g], b[g + 1]) for g in range(world)]
    assert sum(p.shape[1] for p in parts) == e.shape[1]
    for g, p in enumerate(parts):
        assert p[0].min() >= 0 and p[0].max() < b[g + 1] - b[g]


def test_shard_edges_strong_partitions_a_config_graph():
    """Per-rank drawing of a strong-scaled graph (bench.py, configs too large to
    draw on every rank): contiguous user ranges, edges in proportion, unique
    pairs, local ids in range, the same item popularity order on every rank."""
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    import bbgr  # noqa: F401
    from bbgr.synthetic import CONFIGS, shard_edges_strong, user_ranges
    c = CONFIGS["C2"]
    world = 3
    b = user_ranges(c["num_users"], world)
    total, tops = 0, []
    for r in range(world):
        e, lo, hi = shard_edges_strong("C2", r, world)
        assert (lo, hi) == (b[r], b[r + 1])
        assert e.dtype == np.int32 and e.shape[0] == 2
        assert e[0].min() >= 0 and e[0].max() < hi - lo
        assert e[1].min() >= 0 and e[1].max() < c["num_items"]
        keys = e[0].astype(np.int64) * c["num_items"] + e[1]
        assert np.unique(keys).size == keys.size
        total += e.shape[1]
        tops.append(set(np.argsort(-np.bincount(e[1], minlength=c["num_items"]))[:20]))
    assert total == c["num_edges"]
    assert len(tops[0] & tops[1] & tops[2]) >= 10   # one popularity order


def _owner_worker(rank, world, port, out):
    """Item ownership's exchanges (bbgr.distributed.refresh_from_owners /
    gather_owned, the product functions ShardedTrainer calls): every rank holds
    a whole table whose rows it owns are current and the rest stale."""
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    import bbgr  # noqa: F401
    from bbgr.distributed import gather_owned, owner_bounds, refresh_from_owners
    sys.path.insert(0, HERE)
    from _ports import init_worker
    init_worker(rank, world, port)
    I, d = 23, 5
    bounds = owner_bounds(I, world)
    g = torch.Generator().manual_seed(0)
    truth = torch.randn(I, d, generator=g)
    truth[3] = -0.0   # signed zeros and exact bit patterns travel as copies
    stale = truth + 100.0 * (rank + 1)   # every rank's view: stale everywhere ...
    a, b = bounds[rank], bounds[rank + 1]
    stale[a:b] = truth[a:b]               # ... but at the rows it owns
    # (-1: a sampler's "no negative" row, refreshed as row 0)
    rows = torch.tensor([0, 3, 3, I - 1, bounds[1], 7, -1, 11], dtype=torch.int64)
    t = stale.clone()
    refresh_from_owners(t, rows, bounds)
    whole = gather_owned(truth[a:b].contiguous(), bounds)
    np.savez(os.path.join(out, f"own{rank}.npz"), t=t.numpy(), stale=stale.numpy(),
             truth=truth.numpy(), rows=rows.numpy(), whole=whole.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_item_ownership_refresh_and_gather_are_exact(tmp_path, world):
    _spawn(_owner_worker, world, str(tmp_path))
    for k in range(world):
        z = np.load(tmp_path / f"own{k}.npz")
        rows = np.unique(np.clip(z["rows"], 0, None))
        got, want = z["t"], z["stale"].copy()
        want[rows] = z["truth"][rows]          # refreshed rows = the owners' bits
        assert got.tobytes() == want.tobytes()
        assert np.signbit(got[3]).all()        # -0.0 copied, not summed
        assert z["whole"].tobytes() == z["truth"].tobytes()


def test_sharded_item_table_guard_raises_on_stale_rows():
    """ShardedTrainer.item_w: between steps with item
    ownership at N > 1 the rows owned by other ranks lag, so an outside read
    raises (never returns stale rows); the trainer's own methods (step,
    sync_items, forward, state_dict) read it; once current it reads freely."""
    import torch
    from bbgr.distributed import ShardedTrainer, _item_table_owner
    tr = object.__new__(ShardedTrainer)
    t = torch.arange(6.0).reshape(3, 2)
    tr.item_w = t
    tr._items_stale = False
    assert tr.item_w is t
    tr._items_stale = True                       # after an owned-rows Adam at N > 1
    with pytest.raises(RuntimeError, match="sync_items"):
        tr.item_w
    inside = _item_table_owner(lambda self: self.item_w)
    assert inside(tr) is t                       # the trainer's own methods
    with pytest.raises(RuntimeError):            # ... and only while inside
        tr.item_w
    tr._items_stale = False                      # what sync_items() leaves
    assert tr.item_w is t
    for name in ("step", "sync_items", "forward", "state_dict"):
        assert getattr(ShardedTrainer, name).__wrapped__ is not None
