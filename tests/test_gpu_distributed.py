"""GPU: the real ShardedTrainer (HIP kernels + torch.distributed) at world
sizes 2 and 3. RCCL cannot run two ranks on one device, so the ranks share
cuda:0 over the gloo backend; the collective schedule is the one RCCL runs
at round end on 8 GPUs. Checked against the float64 oracle on the union of
the ranks' batches."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("variant,mode,frontier,world,order", [
    ("v2_pop", "strong", "frontier", 2, "input"), ("cu_fair", "strong", "frontier", 2, "input"),
    ("v2_pop", "strong", "dense", 2, "input"), ("v2_pop", "weak", "frontier", 2, "input"),
    ("cu_fair", "weak", "frontier", 2, "input"), ("v2_pop", "strong", "frontier", 3, "input"),
    ("v2_pop", "weak", "frontier", 3, "input"), ("v2_pop", "weak", "frontier", 2, "degree"),
    ("v2_pop", "strong", "frontier", 3, "degree"), ("cu_fair", "weak", "dense", 2, "degree")])
def test_sharded_step_vs_oracle(tmp_path, variant, mode, frontier, world, order):
    """order="degree": every rank numbers its users by local degree and the
    items by GLOBAL degree (identical on every rank); results read back by
    input id."""
    from oracle import ref_numpy as R
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}",
           "--standalone", "--local-addr=127.0.0.1",
           os.path.join(HERE, "dist_worker.py"), str(tmp_path), variant, mode, frontier, order]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    ranks = [dict(np.load(tmp_path / f"rank{k}.npz")) for k in range(world)]
    if mode == "strong":
        g = np.load(os.path.join(HERE, "golden", "golden_small.npz"))
        U, I, E, DUP, D, K, B = (int(x) for x in g["meta"])
        e, cred, u0, i0 = g["edges"], g["cred"], g["u0"], g["i0"]
    else:   # the union of the two shards is the global graph
        sys.path.insert(0, HERE)
        from dist_worker import WEAK_I, WEAK_U
        parts = [np.load(tmp_path / f"edges{k}.npy") + np.array([[k * WEAK_U], [0]], np.int32)
                 for k in range(world)]
        e = np.concatenate(parts, 1)
        U, I, K = world * WEAK_U, WEAK_I, 3
        cred = None
        rng = np.random.default_rng(5)
        u0 = rng.uniform(-1, 1, (U, 64)).astype(np.float32)
        i0 = rng.uniform(-1, 1, (I, 64)).astype(np.float32)
    # replicas of the item side are bitwise identical across ranks
    for r in ranks[1:]:
        np.testing.assert_array_equal(ranks[0]["item_w"], r["item_w"])
        np.testing.assert_array_equal(ranks[0]["g_i0"], r["g_i0"])
    assert ranks[0]["lo"] == 0 and ranks[-1]["hi"] == U
    assert all(ranks[k]["hi"] == ranks[k + 1]["lo"] for k in range(world - 1))
    users = np.concatenate([r["users"] for r in ranks])
    pos = np.concatenate([r["pos"] for r in ranks])
    neg = np.concatenate([r["neg"] for r in ranks])
    if variant == "cu_fair":
        A, Bm, deg_i = R.j_mats(e, U, I, cred)
        uf, itf, _, _ = R.propagate_j(A, Bm, u0, i0, K)
        pop, lam = deg_i / max(deg_i.max(), 1.0), 0.05
    else:
        A, Bm = R.gs_mats(e, U, I, cred)
        uf, itf, _, _ = R.propagate_gs(A, Bm, u0, i0, K)
        pop, lam = None, 0.0
    loss, gr = R.bpr_loss(uf, itf, u0, i0, users, pos, neg, 1e-4, pop, lam)
    if variant == "cu_fair":
        gu0, gi0 = R.backward_j(A, Bm, gr["g_uf"], gr["g_if"], K)
    else:
        gu0, gi0 = R.backward_gs(A, Bm, gr["g_uf"], gr["g_if"], K)
    gu0, gi0 = gu0 + gr["g_ue"], gi0 + gr["g_ie"]

    def close(got, ref, what, tol=1e-5):
        err = np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30)
        assert err <= tol, f"{what}: {err:.3e}"

    if frontier == "dense":   # frontier mode leaves non-batch final rows stale
        close(np.concatenate([r["uf"] for r in ranks]), uf, "u_final")
        close(ranks[0]["itf"], itf, "i_final")
    else:
        bu = users
        close(np.concatenate([r["uf"] for r in ranks])[bu], uf[bu], "u_final @ batch")
        bi = np.concatenate([pos, neg])
        close(ranks[0]["itf"][bi], itf[bi], "i_final @ batch")
    close(np.concatenate([r["g_u0"] for r in ranks]), gu0, "grad u0")
    close(ranks[0]["g_i0"], gi0, "grad i0")
    assert abs(ranks[0]["loss"] - loss) <= 1e-5 * loss


@pytest.mark.parametrize("variant", ["v2_pop", "cu_fair"])
def test_sharded_fused_adam_and_sparse_exchange(tmp_path, variant):
    """Fused Adam (user Adam in the last backward SpMM, item Adam on the sparse
    gradient) == separate gradient + Adam, and the frontier-row (compacted)
    exchange == the dense item-table exchange, over three sharded steps."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--standalone", "--local-addr=127.0.0.1",
           os.path.join(HERE, "dist_worker.py"), str(tmp_path), variant, "fused"]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    ranks = [dict(np.load(tmp_path / f"fused{k}.npz")) for k in range(2)]
    for rk in ranks:
        assert bool(rk["fused_dense_fused"]) == (variant == "v2_pop")
        for fuse in ("sep", "fused"):
            # the compact exchange sums the same values in the same order (gloo, 2 ranks)
            for key in ("user_w", "item_w", "m_i", "loss"):
                np.testing.assert_array_equal(rk[f"{fuse}_sparse_{key}"],
                                              rk[f"{fuse}_dense_{key}"])
        for key in ("user_w", "item_w"):
            a, b = rk[f"fused_sparse_{key}"], rk[f"sep_sparse_{key}"]
            err = np.linalg.norm(a - b) / np.linalg.norm(b)
            assert err < 1e-6, (key, err)
        np.testing.assert_allclose(rk["fused_sparse_loss"], rk["sep_sparse_loss"], rtol=1e-6)
    for key in ("sep_sparse_item_w", "fused_sparse_item_w", "fused_sparse_m_i"):
        np.testing.assert_array_equal(ranks[0][key], ranks[1][key])   # replicas identical
    for rk in ranks:   # item Adam beside the chain (default at N > 1) == in the chain
        for key in ("user_w", "item_w", "m_i", "loss"):
            np.testing.assert_array_equal(rk[f"fused_sparse_{key}"], rk[f"inchain_{key}"])
            # item rows owned by ranks (the fused default) == every rank updating
            # every item row, bit for bit (the next batch's rows refreshed from
            # their owners between steps)
            if variant == "v2_pop":
                np.testing.assert_array_equal(rk[f"fused_sparse_{key}"],
                                              rk[f"replicated_{key}"])
    for rk in ranks:   # the stale-row guard
        own = variant == "v2_pop"   # item ownership: GS with the fused Adam
        assert int(rk["stale_guard"]) == (1 if own else 2)
        np.testing.assert_array_equal(rk["inchain_item_w_attr"], rk["inchain_item_w"])
        if own:
            np.testing.assert_array_equal(rk["inchain_item_w_attr"], rk["replicated_item_w"])
    # two column chains (column_chains=2): the same step over two 32-column
    # slices on their own streams and groups; narrow rows sum in slot order,
    # so equal to rounding, and replicas still bitwise identical
    for rk in ranks:
        for fuse in ("sep", "fused"):
            for key in ("user_w", "item_w"):
                a, b = rk[f"chains_{fuse}_{key}"], rk[f"{fuse}_sparse_{key}"]
                err = np.linalg.norm(a - b) / np.linalg.norm(b)
                assert err < 1e-6, (fuse, key, err)
            np.testing.assert_allclose(rk[f"chains_{fuse}_loss"], rk[f"{fuse}_sparse_loss"],
                                       rtol=1e-6)
    for fuse in ("sep", "fused"):
        np.testing.assert_array_equal(ranks[0][f"chains_{fuse}_item_w"],
                                      ranks[1][f"chains_{fuse}_item_w"])


@pytest.mark.parametrize("variant,order", [("v2_pop", "input"), ("cu_fair", "input"),
                                           ("v2_pop", "degree")])
def test_sharded_trainer_over_rccl_single_rank_matches_fused(tmp_path, variant, order):
    """The sharded step with its collectives on RCCL (world size 1: the one
    RCCL configuration a 1-GPU box can run) equals the single-GPU step."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--standalone", "--local-addr=127.0.0.1",
           os.path.join(HERE, "dist_worker.py"), str(tmp_path), variant, "rccl1", "frontier",
           order]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    z = dict(np.load(tmp_path / "rccl1.npz"))
    np.testing.assert_allclose(z["sharded_loss"], z["single_loss"], rtol=1e-6)
    for key in ("user_w", "item_w", "m_u", "uf", "itf"):
        a, b = z[f"sharded_{key}"], z[f"single_{key}"]
        err = np.linalg.norm(a - b) / np.linalg.norm(b)
        assert err < 1e-6, (key, err)
        # the C ABI's own RCCL communicator (bbgr_allreduce_items) == torch's,
        # on its comm stream and with every collective inline on the compute stream
        np.testing.assert_array_equal(z[f"native_{key}"], z[f"sharded_{key}"])
        np.testing.assert_array_equal(z[f"inline_{key}"], z[f"sharded_{key}"])
        # two interleaved column chains on their own streams, through torch's
        # collectives and through the C ABI's communicator (shared by the chains)
        for tag in ("chains", "chains_native"):
            err = np.linalg.norm(z[f"{tag}_{key}"] - b) / np.linalg.norm(b)
            assert err < 1e-6, (tag, key, err)
    np.testing.assert_allclose(z["chains_loss"], z["single_loss"], rtol=1e-6)
    np.testing.assert_allclose(z["chains_native_loss"], z["single_loss"], rtol=1e-6)
    np.testing.assert_array_equal(z["native_loss"], z["sharded_loss"])
    np.testing.assert_array_equal(z["inline_loss"], z["sharded_loss"])


@pytest.mark.parametrize("variant,frontier,order,world", [
    ("v2_pop", "frontier", "degree", 2), ("cu_fair", "frontier", "input", 2),
    ("v2_pop", "dense", "input", 4)])
def test_column_sharded_step_matches_single_gpu(tmp_path, variant, frontier, order, world):
    """Column (embedding-dimension) sharding, `world` gloo ranks on one device:
    the same batches, losses and full-width tables (all-gathered column slices)
    as the single-GPU trainer after three steps. Not bitwise: the BPR dot
    products are summed per shard then across shards, and narrow rows (64/4 =
    16 columns) sum their edges in slot order."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--standalone", "--local-addr=127.0.0.1",
           os.path.join(HERE, "dist_worker.py"), str(tmp_path), variant, "columns", frontier,
           order]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    ranks = [dict(np.load(tmp_path / f"columns{k}.npz")) for k in range(world)]
    ref = ranks[0]
    assert [int(rk["c1"]) - int(rk["c0"]) for rk in ranks] == [64 // world] * world
    for rk in ranks:
        np.testing.assert_array_equal(rk["users"], ref["ref_users"])
        np.testing.assert_allclose(rk["loss"], ref["ref_loss"], rtol=2e-6)
        for key in ("user_w", "item_w"):
            a, b = rk[key], ref[f"ref_{key}"]
            err = np.linalg.norm(a - b) / np.linalg.norm(b)
            assert err < 1e-6, (key, err)
        np.testing.assert_array_equal(rk["user_w"], ranks[0]["user_w"])   # same gather


@pytest.mark.parametrize("partition", ["columns", "users", "users+chains"])
def test_bench_two_ranks_on_c2(tmp_path, partition):
    """bench.py's N > 1 path end to end (the driver's multi-GPU run) with both
    partitions (and the user-row partition with two interleaved column chains,
    the N >= 8 default), 2 gloo ranks sharing the device, on C2: one JSON line
    from rank 0 with the whole job's graph and the partition named."""
    chains = partition.endswith("+chains")
    partition = partition.split("+")[0]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--standalone", "--local-addr=127.0.0.1",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "C2", "--steps", "3",
           "--warmup", "1", "--dense-check", "1", "--frontier", "on", "--partition", partition,
           "--weak-beside", "2", "--partition-beside", "0", "--chain-beside", "0"] + \
        (["--column-chains", "2"] if chains else [])
    env = dict(os.environ, OMP_NUM_THREADS="4", BBGR_DIST_BACKEND="gloo")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["scaling"] == "strong" and j["partition"] == partition
    assert j["config"]["num_edges"] == 1_000_000 and j["value"] > 0
    assert j["roofline"]["bound"] == "hbm" and j["dense_ms_per_step"] > 0
    if chains:
        assert "2 column chains, 1 item-row ranges" in j["config"]["parallelism"]
    assert j["weak_beside"]["num_edges"] == 2_000_000   # every strong partition
    assert j["partition_beside"] is None


def test_bench_two_ranks_survives_a_failed_beside_run(tmp_path):
    """A beside run that fails on every rank (here injected into the user-row
    runs: an RCCL communicator that will not come up would fail the same way)
    does not cost the line: the ranks agree on it, the line is the run that
    finished, and the failures are listed in beside_errors."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--standalone", "--local-addr=127.0.0.1",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "C2", "--steps", "2",
           "--warmup", "1", "--dense-check", "0", "--frontier", "on", "--weak-beside", "0",
           "--partition", "columns"]
    env = dict(os.environ, OMP_NUM_THREADS="4", BBGR_DIST_BACKEND="gloo",
               BBGR_BENCH_FAIL_BESIDE="users")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    j = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert j["partition"] == "columns" and j["value"] > 0
    assert j["partition_beside"] is None and j["chain_beside"] is None
    assert len(j["beside_errors"]) == 2 and all("injected" in e for e in j["beside_errors"])


def test_bench_two_ranks_survives_a_failed_main_run(tmp_path):
    """The main run failing on every rank (injected; on a real node: a C ABI
    communicator that will not come up for the chain setting the probe chose)
    falls back to the runs beside it: the line is the fastest run that
    finished and the main run's failure is listed in beside_errors."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--standalone", "--local-addr=127.0.0.1",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "C2", "--steps", "2",
           "--warmup", "1", "--dense-check", "0", "--frontier", "on", "--weak-beside", "0",
           "--partition", "users"]
    env = dict(os.environ, OMP_NUM_THREADS="4", BBGR_DIST_BACKEND="gloo",
               BBGR_BENCH_FAIL_BESIDE="main")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    j = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert j["value"] > 0
    assert len(j["beside_errors"]) == 1 and "injected" in j["beside_errors"][0]
    assert j["beside_errors"][0].startswith("users")


def test_bench_sharded_single_rank_with_inline_collectives(tmp_path):
    """bench.py's user-row step at world size 1 over RCCL (--sharded) with
    every collective inline on the compute stream (--native-comm inline): one
    chain, no ranges, a JSON line with the step's value."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--standalone", "--local-addr=127.0.0.1",
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--sharded", "--config", "C2",
           "--steps", "3", "--warmup", "1", "--dense-check", "0", "--frontier", "on",
           "--native-comm", "inline", "--no-cpu-baseline", "--no-torch-reference"]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    j = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert j["value"] > 0 and j["config"]["num_edges"] == 1_000_000
    assert "1 item-row ranges" in j["config"]["parallelism"]
    assert "(inline)" in j["config"]["parallelism"]


def test_bench_two_ranks_measures_both_partitions(tmp_path):
    """--partition-beside (the N > 1 default): the other partition of the same
    graph is timed the same way in the same run; the faster is the line and the
    other is reported beside it."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--standalone", "--local-addr=127.0.0.1",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "C2", "--steps", "3",
           "--warmup", "1", "--dense-check", "1", "--frontier", "on", "--weak-beside", "0"]
    env = dict(os.environ, OMP_NUM_THREADS="4", BBGR_DIST_BACKEND="gloo")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    j = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    b = j["partition_beside"]
    assert {j["partition"], b["part"]} == {"columns", "users"}
    assert j["ms_per_step"] <= b["ms_per_step"] and b["E"] == 1_000_000
    assert j["weak_beside"] is None and j["dense_ms_per_step"] > 0
    # --chain-beside (default): the user-row step in both chain settings — the
    # default (1 chain, 4 ranges over gloo at N = 2) and the one-chain inline
    # schedule — the slower reported beside, the faster named in it
    c = j["chain_beside"]
    assert c["part"] == "users" and c["E"] == 1_000_000
    assert c["chain_mode"] != c["faster_chain_mode"]
    assert c["faster_users_ms_per_step"] <= c["ms_per_step"]
    assert "1 item-row range" in c["chain_mode"] + c["faster_chain_mode"]
    assert "gloo" in c["backend_note"]
    users_ms = (j["ms_per_step"] if j["partition"] == "users" else b["ms_per_step"])
    assert users_ms == c["faster_users_ms_per_step"]
    # the item all-reduce timed alone before the steps (dense payload I*d*4 =
    # 12.8 MB at C2, and 16 MB): t_ar and bus bandwidth through torch's group
    # (gloo here: no RCCL communicator, so no C ABI figures)
    p = j["allreduce_probe"]
    assert p["world"] == 2 and p["sizes_bytes"] == [50_000 * 64 * 4, 16 << 20]
    for mb in (12, 16):
        e = p[f"torch_{mb}MB"]
        assert e["t_ar_ms"] > 0 and e["busbw_GBps"] == pytest.approx(e["algbw_GBps"])  # P = 2
    assert not any(k.startswith("cabi_") for k in p)
    assert j["chain_rule"] is None   # constants only for C4 at N = 8
