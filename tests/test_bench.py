"""CPU: bench.py's accounting — the roofline groups (gather / compulsory
models, dominant-kernel selection inputs) and the reference CPU baseline's
sampled timing path on a small graph. No kernel launches."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.fixture(scope="module")
def bench():
    argv, sys.argv = sys.argv, ["bench.py"]
    try:
        import bench as b
    finally:
        sys.argv = argv
    return b


class _Ev:
    def __init__(self, t):
        self.t = t

    def elapsed_time(self, other):
        return other.t - self.t


class _FakeTimer:
    """SpmmTimer.groups() over hand-made records (no torch.cuda)."""

    def __init__(self, records):
        self.records = records

    def groups(self):
        out = {}
        for rows, nnz, d, m, a, b, tr, nc, sig in self.records:
            g = out.setdefault((m, sig, tr, nc, d), [0, 0.0, 0, 0])
            g[0] += 1
            g[1] += a.elapsed_time(b)
            g[2] += rows
            g[3] += nnz
        return out


def test_roofline_groups_models(bench):
    I, U, E, d = 1000, 5000, 50000, 64
    recs = []
    for s in range(2):   # two steps: one item and one user full launch, one masked
        recs.append((I, E, d, "full", _Ev(0.0), _Ev(0.5), I, U, ""))
        recs.append((U, E, d, "full", _Ev(0.0), _Ev(0.25), U, I, ""))
        recs.append((U, E, d, "masked", _Ev(0.0), _Ev(0.1), U, I, "src"))
    counts = {("masked", "src", U, I, d): [4, 4 * 100, 4 * 1000, 4 * 600]}
    gs = bench.roofline_groups(_FakeTimer(recs), counts, steps=2, count_steps=4, n_items=I)
    by = {(g["kind"], g["side"]): g for g in gs}
    item = by[("full", "item<-user")]
    assert item["launches_per_step"] == 1 and item["avg_ms"] == pytest.approx(0.5)
    assert item["gather_model_bytes"] == E * (8 + 4 * d) + I * (4 + 4 * d)
    assert item["compulsory_bytes"] == E * 8 + U * 4 * d + I * (4 + 4 * d)
    assert item["gather_model_GBps"] == pytest.approx(item["gather_model_bytes"] / 0.5e6)
    user = by[("full", "user<-item")]
    # cache-assisted above the guide's measured random-gather ceiling, not 8 TB/s
    assert user["cache_assisted"] == (user["gather_model_GBps"] > bench.HBM_GATHER_CEILING_GBS)
    assert bench.HBM_GATHER_CEILING_GBS < bench.HBM_PEAK_GBS
    m = by[("masked", "user<-item")]
    assert m["masks"] == "src" and m["rows_per_launch"] == 100 and m["edges_gathered_per_launch"] == 600
    assert m["gather_model_bytes"] == 1000 * 8 + 600 * 4 * d + 100 * (4 + 4 * d)


@pytest.mark.parametrize("variant", ["v2_pop", "cu_fair", "plain"])
def test_cpu_baseline_large_path_on_small_graph(bench, variant):
    """The C3 / C4 form end to end on a small graph: ONE whole measured
    reference step of the variant (sampler loop over the full batch, propagate
    + BPR, backward, Adam) on every CPU of the affinity set; whole reference
    steps of the same variant beside, with their spread."""
    import os
    from bbgr.synthetic import synthetic_credibility, synthetic_edges
    U, I, E = 4000, 1000, 40000
    cfg = dict(num_users=U, num_items=I, num_edges=E, emb_dim=16, num_layers=2, batch=256)
    e = synthetic_edges(U, I, E, seed=3, items="zipf")
    r = bench.cpu_baseline(e, cfg, "X", synthetic_credibility(U, 3), variant,
                           whole_steps=("C1",), whole_reps=3, small_edges=0)
    assert r["kind"] == "port" and r["unit"] == "edges/s"
    assert r["cores"] == bench.cpu_threads() and r["step_measured"]
    assert r["cores"] <= r["affinity_cpus"] == len(os.sched_getaffinity(0))
    comp = r["components_s"]
    assert set(comp) == {"sampler", "forward_bpr", "backward", "adam"}
    assert all(v > 0 for v in comp.values())
    assert r["value"] == pytest.approx(4 * 2 * E / sum(comp.values()), rel=1e-9)
    assert np.isfinite(r["loss"]) and 0.0 < r["loss"] < 1.0   # ~ln 2 at xavier init
    w = r["whole_step_s"]["C1"]
    assert w["median"] > 0 and len(w["runs"]) == 3 and w["iqr_rel"] >= 0
    assert ("pop-mix" in r["sample"]) == (variant == "v2_pop")


def test_cpu_baseline_small_config_is_whole_steps(bench):
    """C1 / C2: the baseline IS the whole reference step of the bench's variant
    (C1: lightgcn.py's symmetric model with uniform negatives, --variant plain)."""
    from bbgr.synthetic import CONFIGS, config_edges, synthetic_credibility
    cfg = CONFIGS["C1"]
    r = bench.cpu_baseline(config_edges("C1"), cfg, "C1",
                           synthetic_credibility(cfg["num_users"], 1), "plain", whole_reps=3)
    w = r["whole_step_s"]["C1"]
    assert r["step_s"] == w["median"] and len(w["runs"]) == 3
    assert r["value"] == pytest.approx(4 * cfg["num_layers"] * cfg["num_edges"] / w["median"])
    assert "plain" in r["sample"]


def test_median_uses_returned_interval(bench):
    t, ts = bench._median_s(lambda: 2.0, reps=3, warmup=1)
    assert t == 2.0 and ts == [2.0, 2.0, 2.0]
    assert np.isfinite(bench._median_s(lambda: None, reps=1)[0])


def test_column_shard_widths_and_partition_rule():
    """Column shards are equal widths from the supported set; the bench's auto
    partition takes columns while shards stay >= MIN_AUTO_WIDTH wide."""
    from bbgr.columns import MIN_AUTO_WIDTH, can_shard_columns, column_range
    assert column_range(64, 2, 1) == (32, 64)
    assert column_range(64, 8, 0) == (0, 8)
    assert column_range(256, 8, 7) == (224, 256)
    for bad in ((64, 3, 0), (64, 2, 2), (64, 16, 0), (48, 2, 0)):
        with pytest.raises(ValueError):
            column_range(*bad)
    assert can_shard_columns(64, 4, MIN_AUTO_WIDTH) and not can_shard_columns(64, 8, MIN_AUTO_WIDTH)
    assert can_shard_columns(64, 8) and not can_shard_columns(64, 16)
    assert can_shard_columns(256, 8, MIN_AUTO_WIDTH)


def test_cpu_list_text_and_threads(bench, monkeypatch):
    """The CPU baseline runs on every CPU of the affinity set, capped by the
    job's stated CPU share (OMP_NUM_THREADS); lists print as ranges."""
    import os
    n = len(os.sched_getaffinity(0))
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    assert bench.cpu_threads() == n
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    assert bench.cpu_threads() == 1
    monkeypatch.setenv("OMP_NUM_THREADS", str(n + 100))
    assert bench.cpu_threads() == n
    assert bench._cpu_list_text([0, 1, 2, 3, 8, 10, 11]) == "0-3,8,10-11"
    assert bench._cpu_list_text([5]) == "5"


def test_edges_per_step_weights_column_slices(bench):
    """A launch over d/N columns counts d_launch/d of its edges: two 32-column
    chains (or one 32-column shard per rank of 2) add up to one 64-column pass."""
    full = {("full", "", 1000, 500, 64): [2, 2000, 800, 800]}
    halves = {("full", "", 1000, 500, 32): [4, 4000, 1600, 1600]}
    assert bench.edges_per_step(full, 64, 2) == (400.0, 400.0)
    assert bench.edges_per_step(halves, 64, 2) == (400.0, 400.0)
    masked = {("masked", "src", 1000, 500, 64): [1, 10, 90, 30]}
    assert bench.edges_per_step(masked, 64, 1) == (30.0, 90.0)


def test_chain_rule_from_the_measured_allreduce(bench):
    """at C4, N = 8 one inline chain wins only while the step's
    exchanges take less than the two-chain compute minus the inline compute;
    other configs have no constants and no rule."""
    dense, front = 1_000_000 * 64 * 4, 16 << 20

    def probe(t_dense, t_front, cabi=True):
        p = {"torch_244MB": {"t_ar_ms": t_dense}, "torch_16MB": {"t_ar_ms": t_front}}
        if cabi:
            p.update({"cabi_244MB": {"t_ar_ms": t_dense}, "cabi_16MB": {"t_ar_ms": t_front}})
        return p
    fast = bench.chain_rule(probe(0.05, 0.01), "C4", 8, 3, dense, front)
    assert fast["predicted"] == "inline"
    assert fast["wire_ms"]["inline"] == pytest.approx(4 * 0.05 + 2 * 0.01)
    slow = bench.chain_rule(probe(1.0, 0.1, cabi=False), "C4", 8, 3, dense, front)
    assert slow["predicted"] == "two_chains"
    assert slow["predicted_ms"]["two_chains"] == pytest.approx(4.2)
    assert bench.chain_rule(probe(0.05, 0.01), "C4", 4, 3, dense, front) is None
    assert bench.chain_rule(None, "C4", 8, 3, dense, front) is None
