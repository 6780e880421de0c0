"""GPU: the drop-in's deferred final tables (bbgr.lazy, bbgr::propagate_rows).

The reference's step reads the propagated tables only through bpr_loss at the
batch rows (Version-2/lighgcn_cu_pop.py:858-863). The drop-in's propagate()
defers them: bpr_loss over one call's pair computes the batch rows only, any
other use computes the whole tables. Both must give the dense path's values
bit for bit: the loss, every gradient, the Adam-updated weights, and the
tables a caller reads.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from bbgr import lazy  # noqa: E402
from bbgr import lightgcn_cu_pop as V2  # noqa: E402
from bbgr import lightgcn_cu_pop_long_tail_exposure as MA  # noqa: E402
from bbgr import operators  # noqa: E402
from bbgr.synthetic import synthetic_credibility, synthetic_edges  # noqa: E402

DEV = "cuda"
U, I, E, D, B = 1500, 700, 20000, 64, 512


def _model(K, module=V2, lazy_on=True, seed=0, n_items=I):
    e = synthetic_edges(U, n_items, E, seed=4, items="zipf")
    torch.manual_seed(seed)
    cred = torch.as_tensor(synthetic_credibility(U, 4))
    M_ui, M_iu = module.build_message_passing_mats(e, U, n_items, cred, DEV)
    m = module.LightGCN(U, n_items, D, K, M_ui, M_iu).to(DEV)
    m.lazy_finals = lazy_on
    return m


def _batch(seed):
    g = torch.Generator().manual_seed(seed)
    users = torch.randperm(U, generator=g)[:B].to(DEV)          # the reference's slices
    pos = torch.randint(0, I, (B,), generator=g).to(DEV)
    neg = torch.randint(0, I, (B,), generator=g).to(DEV)
    return users, pos, neg


def _steps(m, batches, opt_cls=torch.optim.Adam):
    """The reference's loop body (Version-2:858-863) over the batches."""
    opt = opt_cls(m.parameters(), lr=1e-3)
    losses = []
    for users, pos, neg in batches:
        user_emb, item_emb = m.get_user_item_emb()
        loss = m.bpr_loss(users, pos, neg, user_emb, item_emb, 1e-4)
        opt.zero_grad()
        loss.backward()
        grads = [p.grad.clone() for p in m.parameters()]
        opt.step()
        losses.append((float(loss), grads))
    return losses


@pytest.mark.parametrize("K", [3, 2, 1, 0])
@pytest.mark.parametrize("order", ["degree", "input"])
def test_deferred_step_is_bitwise_the_dense_step(K, order, monkeypatch):
    """Three reference steps, deferred (rows only) vs dense: losses, gradients
    and weights equal bit for bit — the drop-in graph in degree order with the
    caller's tables in input order (maps), and a graph kept in input order."""
    monkeypatch.setattr(operators, "DROPIN_VERTEX_ORDER", order)
    batches = [_batch(s) for s in range(3)]
    # a repeated user and a negative outside the table (a sampler giving up)
    batches[1][0][5] = batches[1][0][6]
    batches[2][2][3] = -1
    a, b = _model(K, lazy_on=True), _model(K, lazy_on=False)
    ra, rb = _steps(a, batches), _steps(b, batches)
    for (la, ga), (lb, gb) in zip(ra, rb):
        assert la == lb
        for x, y in zip(ga, gb):
            assert torch.equal(x, y)
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.equal(pa, pb)


@pytest.mark.parametrize("order", ["degree", "input"])
def test_deferred_step_fused_marking_is_the_separate_marking(order, monkeypatch):
    """propagate_rows' marking in one launch (bbgr_rows_mark, the default) and
    as the separate launches (BBGR_ROWS_MARK=0): two reference steps, losses,
    gradients and weights equal bit for bit."""
    monkeypatch.setattr(operators, "DROPIN_VERTEX_ORDER", order)
    batches = [_batch(s) for s in range(2)]
    batches[1][0][5] = batches[1][0][6]
    batches[1][2][3] = -1
    out = []
    for v in ("1", "0"):
        monkeypatch.setenv("BBGR_ROWS_MARK", v)
        m = _model(3)
        out.append((_steps(m, batches), [p.detach().clone() for p in m.parameters()]))
    (ra, pa), (rb, pb) = out
    for (la, ga), (lb, gb) in zip(ra, rb):
        assert la == lb
        for x, y in zip(ga, gb):
            assert torch.equal(x, y)
    for x, y in zip(pa, pb):
        assert torch.equal(x, y)


def test_deferred_tables_compute_on_use_and_equal_the_dense_tables():
    a, b = _model(3, lazy_on=True), _model(3, lazy_on=False)
    uf, itf = a.propagate()
    assert isinstance(uf, lazy.DeferredFinal) and isinstance(itf, lazy.DeferredFinal)
    # metadata answers without computing
    assert uf.shape == (U, D) and itf.size(0) == I and uf.dtype == torch.float32
    assert uf.device.type == "cuda" and uf.dim() == 2 and len(itf) == I and uf.requires_grad
    assert uf._pending.out is None
    ru, ri = b.propagate()
    assert torch.equal(uf[torch.arange(U, device=DEV)], ru)    # indexing computes
    assert uf._pending.out is not None
    assert torch.equal(itf.clone(), ri)
    assert type(uf + 0) is torch.Tensor                        # results are plain
    # the computed tables carry the autograd graph of the call
    (uf.sum() + 2 * itf.sum()).backward()
    (ru.sum() + 2 * ri.sum()).backward()
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.equal(pa.grad, pb.grad)
    # no_grad evaluation (the reference's evaluate_*): tables without a graph
    with torch.no_grad():
        ue, ie = a.get_user_item_emb()
        s = ue[:10] @ ie.T
    assert not s.requires_grad
    assert torch.equal(s, (ru[:10] @ ri.T).detach())


@pytest.mark.parametrize("opt_name", ["torch", "fused"])
def test_deferred_tables_read_after_a_weight_update_raise(opt_name):
    """torch.optim.Adam bumps the weights' versions; bbgr.optim.FusedAdam writes
    them through a raw pointer and bumps them itself: either way a deferred
    table read after the step raises instead of using the new weights."""
    from bbgr.optim import FusedAdam
    m = _model(3)
    opt = (torch.optim.Adam if opt_name == "torch" else FusedAdam)(m.parameters(), lr=1e-3)
    users, pos, neg = _batch(0)
    uf, itf = m.get_user_item_emb()
    m.bpr_loss(users, pos, neg, uf, itf, 1e-4).backward()
    opt.step()                                   # the weights change in place
    with pytest.raises(RuntimeError, match="weights changed"):
        uf[0]
    uf2, itf2 = m.get_user_item_emb()            # a new call is current
    assert np.isfinite(float(m.bpr_loss(users, pos, neg, uf2, itf2, 1e-4)))


def test_method_a_module_defers_too():
    """lightgcn_cu_pop_long_tail_exposure (Method-A operators) inherits the
    deferred tables: its step equals its dense step bit for bit."""
    batches = [_batch(s) for s in range(2)]
    a, b = _model(3, MA, lazy_on=True), _model(3, MA, lazy_on=False)
    for (la, ga), (lb, gb) in zip(_steps(a, batches), _steps(b, batches)):
        assert la == lb
        for x, y in zip(ga, gb):
            assert torch.equal(x, y)


@pytest.mark.parametrize("module,K", [(V2, 3), (MA, 3), (V2, 2), (V2, 4)])
def test_fused_backward_adam_matches_the_separate_step(module, K):
    """bbgr.optim.FusedAdam(fuse_backward=True): the reference's loop body
    (Version-2:858-863) unchanged, the optimizer step carried out inside
    loss.backward() by bbgr::bpr_adam_backward (Adam in the last backward
    products' epilogues). Against FusedAdam's separate step on the same
    batches: the same losses at step 1 (same forward), the moments after step 1
    within 1e-6 (the gradient, rounded in another order), the weights after
    three steps normwise, no .grad on the stepped tables, one step per
    backward, and a deferred table read after the step raises."""
    from bbgr.optim import FusedAdam
    batches = [_batch(s) for s in range(3)]
    batches[1][0][5] = batches[1][0][6]   # a repeated user
    a, b = _model(K, module), _model(K, module)
    w0 = [p.detach().clone() for p in b.parameters()]
    oa = FusedAdam(a.parameters(), lr=1e-3, fuse_backward=True)
    ob = FusedAdam(b.parameters(), lr=1e-3)
    for k, (users, pos, neg) in enumerate(batches):
        ls = []
        for m, o in ((a, oa), (b, ob)):
            uf, itf = m.get_user_item_emb()
            loss = m.bpr_loss(users, pos, neg, uf, itf, 1e-4)
            o.zero_grad()
            loss.backward()
            o.step()
            ls.append(float(loss))
        if k == 0:
            assert ls[0] == ls[1]
            for pa, pb in zip(a.parameters(), b.parameters()):
                for x, y in zip(oa.moments(pa), ob.moments(pb)):
                    assert float((x - y).norm() / y.norm()) < 1e-6
        else:
            assert abs(ls[0] - ls[1]) <= 1e-6 * abs(ls[1])
    for pa, pb, p0 in zip(a.parameters(), b.parameters(), w0):
        assert pa.grad is None and int(oa.state[pa]["step"]) == 3
        da, db = pa.detach() - p0, pb.detach() - p0
        assert float((da - db).norm() / db.norm()) < 1e-3
    uf, itf = a.get_user_item_emb()
    a.bpr_loss(*batches[0], uf, itf, 1e-4).backward()   # a fourth step, in the backward
    with pytest.raises(RuntimeError, match="weights changed"):
        uf[0]


def test_fused_backward_adam_falls_back_where_it_does_not_apply():
    """K = 1 (the last products are the first), torch.optim.Adam, or a weight
    outside the optimizer: the usual path, bit for bit the separate step."""
    from bbgr.optim import FusedAdam
    batches = [_batch(s) for s in range(2)]
    a, b = _model(1), _model(1)
    ra = _steps(a, batches, lambda ps, lr: FusedAdam(ps, lr=lr, fuse_backward=True))
    rb = _steps(b, batches, lambda ps, lr: FusedAdam(ps, lr=lr))
    for (la, ga), (lb, gb) in zip(ra, rb):
        assert la == lb and all(torch.equal(x, y) for x, y in zip(ga, gb))
    c = _model(3)
    oc = FusedAdam([c.user_emb.weight], lr=1e-3, fuse_backward=True)   # item table not in it
    uf, itf = c.get_user_item_emb()
    c.bpr_loss(*batches[0], uf, itf, 1e-4).backward()
    assert c.user_emb.weight.grad is not None and c.item_emb.weight.grad is not None
    oc.step()


def test_fused_backward_adam_moments_leave_in_the_callers_order():
    """On the degree-ordered drop-in graph the in-backward step holds the two
    tables' moments in the graph's row order (the fused epilogue streams them,
    only the weight rows go through the row map). state_dict() and moments()
    hand them out in the caller's order: after one step they equal the
    separate step's within 1e-6; a step() outside the backward (a loss that
    read the whole tables) converts them back and continues; a loaded state
    dict restarts in the caller's order and round-trips."""
    from bbgr.optim import FusedAdam
    a, b = _model(3), _model(3)
    oa = FusedAdam(a.parameters(), lr=1e-3, fuse_backward=True)
    ob = FusedAdam(b.parameters(), lr=1e-3)
    users, pos, neg = _batch(0)
    for m, o in ((a, oa), (b, ob)):
        uf, itf = m.get_user_item_emb()
        o.zero_grad()
        m.bpr_loss(users, pos, neg, uf, itf, 1e-4).backward()
        o.step()
    assert len(oa._graph_rows) == 2 and not ob._graph_rows
    sa, sb = oa.state_dict(), ob.state_dict()
    for k in sa["state"]:
        for key in ("exp_avg", "exp_avg_sq"):
            x, y = sa["state"][k][key], sb["state"][k][key]
            assert float((x - y).norm() / y.norm()) < 1e-6, key
    # the internal tables are still graph-ordered (state_dict made copies)
    pa = next(a.parameters())
    assert not torch.equal(oa.state[pa]["exp_avg"], oa.moments(pa)[0])
    users, pos, neg = _batch(1)
    for m, o in ((a, oa), (b, ob)):
        uf, itf = m.get_user_item_emb()
        uf[0]   # the whole tables: bpr_loss takes the usual path, step() steps
        o.zero_grad()
        m.bpr_loss(users, pos, neg, uf, itf, 1e-4).backward()
        assert all(p.grad is not None for p in m.parameters())
        o.step()
    assert not oa._graph_rows
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert int(oa.state[pa]["step"]) == 2
        assert float((pa - pb).norm() / pb.norm()) < 1e-5
        for x, y in zip(oa.moments(pa), ob.moments(pb)):
            assert float((x - y).norm() / y.norm()) < 1e-5
    with pytest.warns(RuntimeWarning, match="another live in-backward FusedAdam"):
        oc = FusedAdam(a.parameters(), lr=1e-3, fuse_backward=True)   # takes them from oa
    oc.load_state_dict(oa.state_dict())
    for pa in a.parameters():
        assert all(torch.equal(x, y) for x, y in zip(oc.moments(pa), oa.moments(pa)))


def test_fused_backward_adam_with_as_many_items_as_users(monkeypatch):
    """num_users == num_items: the ego rows' first-slot tables of the users and
    of the items are two buffers (one launch fills both; a shared buffer sent
    ego-L2 rows to wrong rows). The in-backward step and the
    deferred sparse-ego loss against the dense separate step."""
    from bbgr.optim import FusedAdam
    batches = [_batch(s) for s in range(3)]
    batches[1][0][5] = batches[1][0][6]   # a repeated user
    for bt in batches:                    # items drawn from [0, U) too
        g = torch.Generator().manual_seed(int(bt[0][0]))
        bt[1][:] = torch.randint(0, U, (B,), generator=g).to(DEV)
        bt[2][:] = torch.randint(0, U, (B,), generator=g).to(DEV)
        bt[1][:8] = bt[0][:8]             # item ids equal to user ids of the batch
    # the deferred loss (bpr_loss_sparse_ego's backward) vs the dense ego table
    from bbgr import bpr
    a, b = _model(3, n_items=U), _model(3, n_items=U, lazy_on=False)
    ra = _steps(a, batches)
    monkeypatch.setattr(bpr, "_receives_dense_grad", lambda *x: False)
    rb = _steps(b, batches)
    monkeypatch.undo()
    for (la, ga), (lb, gb) in zip(ra, rb):
        assert la == lb
        for x, y in zip(ga, gb):
            assert torch.equal(x, y)
    # the in-backward Adam vs the separate step
    c, d = _model(3, n_items=U), _model(3, n_items=U)
    w0 = [p.detach().clone() for p in d.parameters()]
    oc = FusedAdam(c.parameters(), lr=1e-3, fuse_backward=True)
    od = FusedAdam(d.parameters(), lr=1e-3)
    for k, (users, pos, neg) in enumerate(batches):
        for m, o in ((c, oc), (d, od)):
            uf, itf = m.get_user_item_emb()
            loss = m.bpr_loss(users, pos, neg, uf, itf, 1e-2)   # a large ego term
            o.zero_grad()
            loss.backward()
            o.step()
        if k == 0:
            for pc, pd in zip(c.parameters(), d.parameters()):
                for x, y in zip(oc.moments(pc), od.moments(pd)):
                    assert float((x - y).norm() / y.norm()) < 1e-6
    for pc, pd, p0 in zip(c.parameters(), d.parameters(), w0):
        dc, dd = pc.detach() - p0, pd.detach() - p0
        assert float((dc - dd).norm() / dd.norm()) < 1e-3


def test_fused_backward_item_tables_bounded_over_streams():
    """The in-backward Adam keeps its two [I, d] item tables per stream; a
    caller stepping on a new stream each time holds at most two sets."""
    from bbgr.optim import FusedAdam
    from bbgr.ops import pair_key
    a = _model(3)
    oa = FusedAdam(a.parameters(), lr=1e-3, fuse_backward=True)
    key = pair_key(a._operator_pair())
    for s in range(4):
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            uf, itf = a.get_user_item_emb()
            oa.zero_grad()
            a.bpr_loss(*_batch(s), uf, itf, 1e-4).backward()
            oa.step()
        torch.cuda.current_stream().wait_stream(st)
        assert torch.ops.bbgr._item_table_sets(key) == min(s + 1, 2)
    assert all(int(oa.state[p]["step"]) == 4 for p in a.parameters())
    assert all(torch.isfinite(p).all() for p in a.parameters())


def test_fused_backward_adam_refuses_a_second_gradient_path():
    """A loss term that reads the weights directly puts a .grad on a table the
    in-backward step already updated: step() raises instead of dropping it."""
    from bbgr.optim import FusedAdam
    a = _model(3)
    oa = FusedAdam(a.parameters(), lr=1e-3, fuse_backward=True)
    uf, itf = a.get_user_item_emb()
    loss = a.bpr_loss(*_batch(0), uf, itf, 1e-4) + 1e-3 * a.user_emb.weight.norm()
    oa.zero_grad()
    loss.backward()
    with pytest.raises(RuntimeError, match="only consumer"):
        oa.step()


def test_fused_backward_adam_master_copies_are_bitwise_the_caller_order_step():
    """FusedAdam(fuse_backward=True, use_masters=True) on the degree-ordered
    drop-in graph keeps graph-ordered master copies of the two weight tables:
    the in-backward Adam
    updates them with the moments and writes the caller's rows (adam_mirror),
    and the next forward gathers them (bbgr::propagate_rows_graph). Against the
    same optimizer without them: losses, weights and moments bit for bit over
    five steps, including a step after an outside in-place write to the
    weights (the copies are stale then and are rebuilt, not used)."""
    from bbgr.optim import FusedAdam
    batches = [_batch(s) for s in range(5)]
    a, b = _model(3), _model(3)
    oa = FusedAdam(a.parameters(), lr=1e-3, fuse_backward=True)
    ob = FusedAdam(b.parameters(), lr=1e-3, fuse_backward=True)
    oa.use_masters, ob.use_masters = True, False
    for k, (users, pos, neg) in enumerate(batches):
        if k == 3:   # an outside write: both models, the same rows
            with torch.no_grad():
                for m in (a, b):
                    m.user_emb.weight[:7] *= 0.5
                    m.item_emb.weight[3] += 0.25
            assert oa.masters([a.user_emb.weight, a.item_emb.weight],
                              [a._pair.io.user_map64, a._pair.io.item_map64]) is None
        ls = []
        for m, o in ((a, oa), (b, ob)):
            uf, itf = m.get_user_item_emb()
            loss = m.bpr_loss(users, pos, neg, uf, itf, 1e-4)
            o.zero_grad()
            loss.backward()
            o.step()
            ls.append(float(loss))
        assert ls[0] == ls[1], k
        if k >= 1:
            assert len(oa._masters) == 2 and not ob._masters
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.equal(pa, pb)
        for x, y in zip(oa.moments(pa), ob.moments(pb)):
            assert torch.equal(x, y)
    ug, ig = oa.masters([a.user_emb.weight, a.item_emb.weight],
                        [a._pair.io.user_map64, a._pair.io.item_map64])
    assert torch.equal(ug, a.user_emb.weight.detach()[a._pair.io.user_map64])
    assert torch.equal(ig, a.item_emb.weight.detach()[a._pair.io.item_map64])


@pytest.mark.parametrize("order", ["degree", "input"])
def test_fused_backward_user_scatter_without_the_sort(order, monkeypatch):
    """bpr_adam_backward's user-row scatters (the BPR rows into gU, the ego
    rows before the user Adam) in first-slot form (bbgr_rows_add_slots, no
    sort) are bitwise the sorted scatter (BBGR_USER_SORT=1): weights and
    moments over four steps with distinct users, a repeated user, and a
    negative outside the table (an invalid triple) whose user recurs later in
    the batch (the invalid slot then leads that user's rows)."""
    from bbgr.optim import FusedAdam
    monkeypatch.setattr(operators, "DROPIN_VERTEX_ORDER", order)
    batches = [_batch(s) for s in range(4)]
    batches[1][0][5] = batches[1][0][6]
    batches[3][2][3] = -1
    batches[3][0][9] = batches[3][0][3]
    out = []
    for sort in ("0", "1"):
        monkeypatch.setenv("BBGR_USER_SORT", sort)
        m = _model(3)
        o = FusedAdam(m.parameters(), lr=1e-3, fuse_backward=True)
        ls = []
        for users, pos, neg in batches:
            uf, itf = m.get_user_item_emb()
            loss = m.bpr_loss(users, pos, neg, uf, itf, 1e-4)
            o.zero_grad()
            loss.backward()
            o.step()
            ls.append(float(loss))
        out.append((ls, [p.detach().clone() for p in m.parameters()],
                    [x.clone() for p in m.parameters() for x in o.moments(p)]))
    assert out[0][0] == out[1][0]
    for x, y in zip(out[0][1] + out[0][2], out[1][1] + out[1][2]):
        assert torch.equal(x, y)
