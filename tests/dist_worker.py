"""Worker for tests/test_gpu_distributed.py (launched by torch.distributed.run):
two gloo ranks share cuda:0 and run one ShardedTrainer step; each rank dumps
its state for the parent test to check against the oracle.

mode "strong": one global graph (the golden fixture) cut into user ranges.
mode "weak":   each rank builds its own user shard over the shared items."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bbgr  # noqa: E402,F401
from bbgr.distributed import ShardedTrainer  # noqa: E402
from bbgr.synthetic import synthetic_edges  # noqa: E402

WEAK_U, WEAK_I, WEAK_E = 200, 150, 2500


def main():
    out_dir, variant, mode = sys.argv[1], sys.argv[2], sys.argv[3]
    frontier = len(sys.argv) < 5 or sys.argv[4] != "dense"
    order = sys.argv[5] if len(sys.argv) > 5 else "input"
    if mode == "fused":
        return fused_vs_separate(out_dir, variant)
    if mode == "rccl1":
        return rccl_single_rank(out_dir, variant, order)
    if mode == "columns":
        return column_sharded(out_dir, variant, frontier, order)
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    torch.cuda.set_device(0)
    lam = 0.05 if variant == "cu_fair" else 0.0
    if mode == "strong":
        g = np.load(os.path.join(ROOT, "tests", "golden", "golden_small.npz"))
        U, I, E, DUP, D, K, B = (int(x) for x in g["meta"])
        tr = ShardedTrainer.from_global_edges(
            g["edges"], U, I, variant, cred=g["cred"], emb_dim=D, num_layers=K, batch_size=64,
            device="cuda:0", u0=g["u0"], i0=g["i0"], lambda_fair=lam, frontier=frontier,
            exchange_parts=3, fuse_adam=False, vertex_order=order)
    else:
        e = synthetic_edges(WEAK_U, WEAK_I, WEAK_E, 100 + rank, items="zipf", item_seed=100)
        rng = np.random.default_rng(5)
        world = dist.get_world_size()
        u0 = rng.uniform(-1, 1, (world * WEAK_U, 64)).astype(np.float32)[rank * WEAK_U:(rank + 1) * WEAK_U]
        i0 = rng.uniform(-1, 1, (WEAK_I, 64)).astype(np.float32)
        np.save(os.path.join(out_dir, f"edges{rank}.npy"), e)
        tr = ShardedTrainer(e, WEAK_U, WEAK_I, variant, emb_dim=64, num_layers=3, batch_size=32,
                            device="cuda:0", u0=u0, i0=i0, lambda_fair=lam,
                            user_offset=rank * WEAK_U, frontier=frontier, exchange_parts=2,
                            fuse_adam=False, vertex_order=order)
    loss = float(tr.step())
    tr.sync_items()                        # item rows owned elsewhere made current
    users, pos, neg = tr.batch()           # input (local) ids
    go, gi = tr.graph.user_order, tr.graph.item_order

    def by_input(order, x):                # internal rows -> rows by input id
        return (x if order is None else order.rows_to_input(x)).cpu().numpy()

    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), lo=tr.lo, hi=tr.hi,
             users=users.cpu().numpy() + tr.lo, pos=pos.cpu().numpy(), neg=neg.cpu().numpy(),
             g_u0=by_input(go, tr.g_u0), g_i0=by_input(gi, tr.g_i0),
             user_w=by_input(go, tr.user_w), item_w=by_input(gi, tr.item_w), loss=loss,
             uf=by_input(go, tr.uf), itf=by_input(gi, tr.itf))
    dist.destroy_process_group()


def fused_vs_separate(out_dir, variant):
    """Three steps of four sharded trainers on the same shards and seeds:
    separate / fused Adam x dense / sparse (frontier-row) exchange."""
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    torch.cuda.set_device(0)
    e = synthetic_edges(WEAK_U, WEAK_I, WEAK_E, 300 + rank, items="zipf", item_seed=300)
    rng = np.random.default_rng(9)
    u0 = rng.uniform(-0.5, 0.5, (2 * WEAK_U, 64)).astype(np.float32)[rank * WEAK_U:(rank + 1) * WEAK_U]
    i0 = rng.uniform(-0.5, 0.5, (WEAK_I, 64)).astype(np.float32)
    out = {}
    for fuse in (False, True):
        for sparse in (False, True):
            tr = ShardedTrainer(e, WEAK_U, WEAK_I, variant, emb_dim=64, num_layers=3,
                                batch_size=32, device="cuda:0", u0=u0, i0=i0,
                                user_offset=rank * WEAK_U, exchange_parts=2, fuse_adam=fuse, frontier=True,
                                sparse_exchange=sparse)
            losses = [float(tr.step()) for _ in range(3)]
            tag = f"{'fused' if fuse else 'sep'}_{'sparse' if sparse else 'dense'}"
            items = tr.sync_items()   # (item ownership: rows and moments from the owners)
            out[f"{tag}_user_w"] = tr.user_w.cpu().numpy()
            out[f"{tag}_item_w"] = items["item_w"].cpu().numpy()
            out[f"{tag}_m_i"] = items["m_i"].cpu().numpy()
            out[f"{tag}_loss"] = np.array(losses)
            out[f"{tag}_fused"] = np.array(tr.fuse_adam)
    # the item Adam in the chain instead of on the side stream (world 2
    # overlaps it by default): bitwise the same step
    tr = ShardedTrainer(e, WEAK_U, WEAK_I, variant, emb_dim=64, num_layers=3, batch_size=32,
                        device="cuda:0", u0=u0, i0=i0, user_offset=rank * WEAK_U,
                        exchange_parts=2, fuse_adam=True, frontier=True, overlap_item_adam=False)
    losses = [float(tr.step()) for _ in range(3)]
    # between steps, rows owned by the other rank lag: reading the table raises
    # (1) instead of returning them; without ownership it reads (2)
    try:
        tr.item_w
        out["stale_guard"] = np.array(2)
    except RuntimeError:
        out["stale_guard"] = np.array(1)
    items = tr.sync_items()
    out["inchain_item_w_attr"] = tr.item_w.cpu().numpy()   # current after sync_items()
    out["inchain_user_w"] = tr.user_w.cpu().numpy()
    out["inchain_item_w"] = items["item_w"].cpu().numpy()
    out["inchain_m_i"] = items["m_i"].cpu().numpy()
    out["inchain_loss"] = np.array(losses)
    # the replicated item Adam (own_items=False): every rank updates every item
    # row; bitwise the owned-rows step after the owners' rows are gathered
    tr = ShardedTrainer(e, WEAK_U, WEAK_I, variant, emb_dim=64, num_layers=3, batch_size=32,
                        device="cuda:0", u0=u0, i0=i0, user_offset=rank * WEAK_U,
                        exchange_parts=2, fuse_adam=True, frontier=True, own_items=False)
    losses = [float(tr.step()) for _ in range(3)]
    out["replicated_user_w"] = tr.user_w.cpu().numpy()
    out["replicated_item_w"] = tr.item_w.cpu().numpy()
    out["replicated_m_i"] = tr.m_i.cpu().numpy()
    out["replicated_loss"] = np.array(losses)
    # two column chains (32 columns each, own streams and exchange groups)
    for fuse in (False, True):
        tr = ShardedTrainer(e, WEAK_U, WEAK_I, variant, emb_dim=64, num_layers=3,
                            batch_size=32, device="cuda:0", u0=u0, i0=i0,
                            user_offset=rank * WEAK_U, exchange_parts=2, fuse_adam=fuse,
                            frontier=True, column_chains=2)
        losses = [float(tr.step()) for _ in range(3)]
        tag = f"chains_{'fused' if fuse else 'sep'}"
        out[f"{tag}_user_w"] = tr.user_w.cpu().numpy()
        out[f"{tag}_item_w"] = tr.sync_items()["item_w"].cpu().numpy()
        out[f"{tag}_loss"] = np.array(losses)
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"fused{rank}.npz"), **out)
    dist.destroy_process_group()


def rccl_single_rank(out_dir, variant, order="input"):
    """World size 1 over RCCL ("nccl"): the sharded trainer's collectives run
    through RCCL itself (uint8 / fp32 all-reduce, async ranges, all-gather of
    int64 and fp32) and its steps must equal the single-GPU FusedTrainer's."""
    from bbgr.graph import BipartiteGraph
    from bbgr.trainer import FusedTrainer
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    U, I, E = 3000, 1200, 40000
    e = synthetic_edges(U, I, E, 77, items="zipf")
    rng = np.random.default_rng(3)
    u0 = rng.uniform(-0.5, 0.5, (U, 64)).astype(np.float32)
    i0 = rng.uniform(-0.5, 0.5, (I, 64)).astype(np.float32)
    kw = dict(emb_dim=64, num_layers=3, batch_size=256, u0=u0, i0=i0, frontier=True)
    sh = ShardedTrainer(e, U, I, variant, device="cuda:0", exchange_parts=3,
                        vertex_order=order, **kw)
    one = FusedTrainer(BipartiteGraph(e, U, I, "cuda:0", vertex_order=order), variant, **kw)
    nat = ShardedTrainer(e, U, I, variant, device="cuda:0", exchange_parts=3,
                         vertex_order=order, native_comm=True, **kw)   # bbgr_allreduce_items
    chains = ShardedTrainer(e, U, I, variant, device="cuda:0", exchange_parts=3,
                            vertex_order=order, column_chains=2, **kw)   # interleaved chains
    chains_nat = ShardedTrainer(e, U, I, variant, device="cuda:0", exchange_parts=1,
                                vertex_order=order, column_chains=2, native_comm=True, **kw)
    # every collective of the step on the compute stream (bbgr_comm_allreduce /
    # _allgather / bbgr_allreduce_items inline)
    inl = ShardedTrainer(e, U, I, variant, device="cuda:0", exchange_parts=3,
                         vertex_order=order, native_comm="inline", **kw)
    out = {}
    for tag, tr in (("sharded", sh), ("single", one), ("native", nat), ("chains", chains),
                    ("chains_native", chains_nat), ("inline", inl)):
        out[f"{tag}_loss"] = np.array([float(tr.step()) for _ in range(3)])
        out[f"{tag}_user_w"] = tr.user_w.cpu().numpy()
        out[f"{tag}_item_w"] = tr.item_w.cpu().numpy()
        out[f"{tag}_m_u"] = tr.m_u.cpu().numpy()
        uf, itf = tr.forward()   # sharded: collective, item sums exchanged
        out[f"{tag}_uf"], out[f"{tag}_itf"] = uf.cpu().numpy(), itf.cpu().numpy()
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, "rccl1.npz"), **out)
    nat.close()   # bbgr_comm_destroy
    chains_nat.close()
    inl.close()
    dist.destroy_process_group()


def column_sharded(out_dir, variant, frontier, order):
    """Column (embedding-dimension) sharding: each rank holds the whole graph
    and d/world columns; three steps, then the full-width tables (all-gathered)
    and the losses, with rank 0's single-GPU FusedTrainer on the same inputs."""
    from bbgr.columns import ColumnShardedTrainer
    from bbgr.graph import BipartiteGraph
    from bbgr.synthetic import synthetic_credibility
    from bbgr.trainer import FusedTrainer
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    U, I, E = 3000, 900, 40000
    e = synthetic_edges(U, I, E, 21, items="zipf")
    rng = np.random.default_rng(21)
    u0 = rng.uniform(-0.3, 0.3, (U, 64)).astype(np.float32)
    i0 = rng.uniform(-0.3, 0.3, (I, 64)).astype(np.float32)
    kw = dict(cred=synthetic_credibility(U, 21), emb_dim=64, num_layers=3, batch_size=512,
              u0=u0, i0=i0, frontier=frontier,
              lambda_fair=0.05 if variant == "cu_fair" else 0.0)
    tr = ColumnShardedTrainer(e, U, I, variant, device="cuda:0", vertex_order=order, **kw)
    losses = [float(tr.step()) for _ in range(3)]
    sd = tr.full_state_dict()
    out = {"loss": np.array(losses), "c0": np.array(tr.c0), "c1": np.array(tr.c1),
           "user_w": sd["user_emb.weight"].cpu().numpy(),
           "item_w": sd["item_emb.weight"].cpu().numpy(),
           "users": tr.batch()[0].cpu().numpy()}
    if rank == 0:
        one = FusedTrainer(BipartiteGraph(e, U, I, "cuda:0", vertex_order=order), variant, **kw)
        out["ref_loss"] = np.array([float(one.step()) for _ in range(3)])
        rsd = one.state_dict()
        out["ref_user_w"] = rsd["user_emb.weight"].cpu().numpy()
        out["ref_item_w"] = rsd["item_emb.weight"].cpu().numpy()
        out["ref_users"] = one.batch()[0].cpu().numpy()
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"columns{rank}.npz"), **out)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
