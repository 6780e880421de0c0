"""GPU: the graph-capturable training step.

* device step state (bbgr_step_begin / bbgr_sample_dev / bbgr_adam_dev and the
  fused Adam's adam_state): an eager step reading t and the sampler counter
  from device memory is bitwise the host-scalar step;
* GraphedStep (torch.cuda.CUDAGraph capture of FusedTrainer._step): replays
  are bitwise the eager steps, across an epoch boundary and for the fused
  GS / Jacobi Adam and the separate Adam;
* in-launch split-row reduction: the arrival counters of the partial
  workspace are zero again after every launch, and results are bitwise
  stable across launches.
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from bbgr.graph import BipartiteGraph  # noqa: E402
from bbgr.synthetic import synthetic_credibility, synthetic_edges  # noqa: E402
from bbgr.propagate import ORDER_GS  # noqa: E402
from bbgr.trainer import FusedTrainer, GraphedStep  # noqa: E402

DEV = "cuda"


def _graph(U=3000, I=1200, E=60000, seed=5):
    e = synthetic_edges(U, I, E, seed=seed, items="zipf")
    return e, BipartiteGraph(e, U, I, DEV, vertex_order="degree")


def _state(tr):
    return [tr.user_w, tr.item_w, tr.m_u, tr.v_u, tr.m_i, tr.v_i]


def _assert_same(a, b):
    for x, y in zip(_state(a), _state(b)):
        assert torch.equal(x, y)
    assert a.step_count == b.step_count and a.sampler.counter == b.sampler.counter


@pytest.mark.parametrize("variant,fuse", [("v2_pop", True), ("cu_fair", True),
                                          ("v2_pop", False)])
def test_device_state_eager_matches_host_scalars(variant, fuse):
    e, g = _graph()
    kw = dict(cred=synthetic_credibility(3000, 5), emb_dim=64, num_layers=3, batch_size=256,
              frontier=True, fuse_adam=fuse, seed=3)
    a, b = FusedTrainer(g, variant, **kw), FusedTrainer(g, variant, **kw)
    b.enable_device_state()
    for _ in range(4):
        assert float(a.step()) == float(b.step())
    _assert_same(a, b)
    st = b.dev_state.state.cpu().tolist()
    assert st == [4, 3, 4, b.dev_state.max_steps]   # t, this counter, next counter, table


@pytest.mark.parametrize("variant,fuse,frontier", [("v2_pop", True, True),
                                                   ("v2_pop", True, False),
                                                   ("cu_fair", True, True),
                                                   ("v2_pop", False, True)])
def test_graphed_step_replays_bitwise_eager(variant, fuse, frontier):
    """Captured once, replayed: weights, Adam moments, loss and batch are the
    eager trainer's bit for bit, also across epoch boundaries (3000 users,
    batch 700: the permutation is redrawn every 5th step; the short tail runs
    eagerly)."""
    e, g = _graph()
    kw = dict(cred=synthetic_credibility(3000, 5), emb_dim=64, num_layers=3, batch_size=700,
              frontier=frontier, fuse_adam=fuse, seed=11)
    a, b = FusedTrainer(g, variant, **kw), FusedTrainer(g, variant, **kw)
    gs = GraphedStep(b)                        # runs b's first step eagerly
    la = [float(a.step())]
    lb = [float(gs.first_loss)]
    for _ in range(11):
        la.append(float(a.step()))
        lb.append(float(gs.step()))
        ua, pa, na = a.batch()
        ub, pb, nb = b.batch()
        assert torch.equal(ua, ub) and torch.equal(pa, pb) and torch.equal(na, nb)
    assert la == lb
    _assert_same(a, b)
    assert a.epoch >= 3


def test_graphed_step_sparse_tables_stay_zero():
    """The replayed step restores the all-zero invariant of its sparse
    gradient tables and masks, as the eager step does."""
    e, g = _graph()
    tr = FusedTrainer(g, "v2_pop", emb_dim=64, num_layers=2, batch_size=512, frontier=True)
    gs = GraphedStep(tr)
    for _ in range(3):
        gs.step()
    torch.cuda.synchronize()
    assert float(tr.g_uf.abs().sum()) == 0.0 and float(tr.g_if.abs().sum()) == 0.0
    assert int(tr.mask_u.sum()) == 0 and int(tr.mask_i.sum()) == 0


def test_split_rows_finish_in_launch_and_counters_reset():
    """Rows cut into several chunks are summed by their last-arriving chunk in
    the same launch: the arrival counters behind the partials are zero after
    each launch and repeated launches give bitwise identical tables."""
    from bbgr import propagate as P
    U, I = 4000, 300
    e = synthetic_edges(U, I, 200000, seed=9, items="zipf")   # hub items: deg >> 2048
    g = BipartiteGraph(e, U, I, DEV)
    prod = P.Product(g.item_csr, None, None, None, {})
    assert g.item_csr.n_split > 0
    x = torch.randn(U, 64, device=DEV)
    outs = []
    for _ in range(3):
        y = torch.empty(I, 64, device=DEV)
        P.spmm(prod, x, False, y=y)
        outs.append(y)
        ws = prod.workspace(64)
        cnt = ws[g.item_csr.n_chunks * 64:].view(torch.int32)
        torch.cuda.synchronize()
        assert int(cnt.abs().sum()) == 0
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])
    # the launch computes the plain sum over each row's edges (weight_mode 0,
    # no scales): against float64
    A = torch.zeros(I, U, dtype=torch.float64)
    ii, uu = torch.as_tensor(e[1], dtype=torch.long), torch.as_tensor(e[0], dtype=torch.long)
    A.index_put_((ii, uu), torch.ones(ii.numel(), dtype=torch.float64), accumulate=True)
    ref = (A @ x.double().cpu()).numpy()
    got = outs[0].double().cpu().numpy()
    assert np.linalg.norm(got - ref) <= 1e-5 * np.linalg.norm(ref)


def test_transpose_slots_map_every_edge_once():
    """bbgr_transpose_slots: every user-CSR slot maps to the item-CSR slot of
    the same edge (duplicates: k-th copy to k-th copy), a permutation."""
    U, I = 2000, 300
    e = synthetic_edges(U, I, 40000, 6, items="zipf", duplicates=300)
    g = BipartiteGraph(e, U, I, "cuda", vertex_order="degree")
    t = g.user_item_slots().long().cpu()
    uc_ptr, uc_idx = g.user_csr.indptr.long().cpu(), g.user_csr.indices.long().cpu()
    ic_ptr, ic_idx = g.item_csr.indptr.long().cpu(), g.item_csr.indices.long().cpu()
    E = uc_idx.numel()
    assert torch.equal(torch.sort(t).values, torch.arange(E))
    urow = torch.repeat_interleave(torch.arange(U), uc_ptr[1:] - uc_ptr[:-1])
    irow = torch.repeat_interleave(torch.arange(I), ic_ptr[1:] - ic_ptr[:-1])
    assert torch.equal(ic_idx[t], urow) and torch.equal(irow[t], uc_idx)
    # the map built from the CSR builds' permutations (user_item_slots) is
    # bitwise the per-edge binary search's (bbgr_transpose_slots)
    import ctypes
    from bbgr._lib import call, ptr, stream_handle
    ts = torch.empty(max(E, 1), dtype=torch.int32, device="cuda")
    call("bbgr_transpose_slots", ctypes.byref(g.user_csr._struct),
         ctypes.byref(g.item_csr._struct), ptr(ts), stream_handle())
    assert torch.equal(ts[:E].long().cpu(), t[:E])


@pytest.mark.parametrize("variant,bits,listed", [("v2_pop", True, True),
                                                 ("cu_fair", True, True),
                                                 ("v2_pop", True, False),
                                                 ("v2_pop", False, True)])
def test_slot_bitmap_first_item_product_is_bitwise_the_mask(variant, bits, listed):
    """The first backward item product tests liveness on the batch users' slot
    bitmap (bbgr_spmm_args.src_bits; single-chunk hub rows then summed by one
    lane group in the chunk workgroup's order) instead of scanning indices,
    and visits the frontier through the row list the masking built
    (bbgr_mark_list, device length): weights, moments and losses over three
    steps equal the mask-only trainer bit for bit (hub items: chunked and
    split rows), and the bitmap and list count are zero again after every
    step."""
    U, I = 20000, 3000
    e = synthetic_edges(U, I, 300000, 8, items="zipf")
    g = BipartiteGraph(e, U, I, "cuda", vertex_order="degree")
    kw = dict(cred=synthetic_credibility(U, 8), emb_dim=64, num_layers=3, batch_size=2048,
              frontier=True, seed=5)
    a, b = FusedTrainer(g, variant, **kw), FusedTrainer(g, variant, **kw)
    assert a.slot_bits is not None
    assert (a.item_list is not None) == (a.order == ORDER_GS)   # the list: GS only
    listed = listed and a.item_list is not None
    if not bits:
        a.slot_bits = a.slot_map = None
    if not listed:
        a.item_list = None
    b.slot_bits = b.slot_map = None          # the mask-only path
    b.item_list = None
    for _ in range(3):
        assert float(a.step()) == float(b.step())
        if bits:
            assert int(a.slot_bits.abs().sum()) == 0
        if listed:
            assert int(a.item_count.item()) == 0
    for x, y in ((a.user_w, b.user_w), (a.item_w, b.item_w), (a.m_u, b.m_u), (a.v_i, b.v_i)):
        assert torch.equal(x, y)


@pytest.mark.parametrize("fuse,K", [(True, 3), (False, 3), (True, 2)])
def test_tagged_user_indices_step_is_bitwise_the_mask_step(fuse, K, monkeypatch):
    """GS with the frontier: the first forward user product writes the user
    CSR's indices tagged with the item frontier and the first backward user
    product reads them (bbgr_spmm_args.tag_out / src_tagged) instead of the
    mask byte per edge: losses, weights and moments equal the mask step's bit
    for bit over five steps (BBGR_TAGGED=1 turns it on; the default keeps the
    mask)."""
    e, g = _graph()
    kw = dict(cred=synthetic_credibility(3000, 5), emb_dim=64, num_layers=K, batch_size=256,
              frontier=True, fuse_adam=fuse, seed=7)
    b = FusedTrainer(g, "v2_pop", **kw)
    monkeypatch.setenv("BBGR_TAGGED", "1")
    a = FusedTrainer(g, "v2_pop", **kw)
    assert a.tagged is not None and b.tagged is None
    for _ in range(5):
        assert float(a.step()) == float(b.step())
    _assert_same(a, b)
    # the copy holds this step's frontier: bit 31 exactly off the item mask
    uc = g.user_csr
    a._set_masks(a._last_users, a.pos, a.neg, 1)
    idx = uc.indices[:uc.nnz].long()
    live = a.mask_i[idx].bool()
    a._set_masks(a._last_users, a.pos, a.neg, 0)
    want = torch.where(live, idx, idx | (1 << 31)).to(torch.int64) & 0xFFFFFFFF
    assert torch.equal(a.tagged[:uc.nnz].to(torch.int64) & 0xFFFFFFFF, want)


@pytest.mark.parametrize("fuse,K,dim", [(True, 3, 64), (False, 3, 64), (True, 2, 64),
                                        (True, 1, 64), (True, 3, 32)])
def test_fused_batch_bookkeeping_is_bitwise_the_separate_launches(fuse, K, dim, monkeypatch):
    """GS frontier: bbgr_batch_begin / bbgr_batch_end (masks, item list, slot
    bits and the sparse gradient rows' reset in one launch each) give the
    separate launches' losses, weights and moments bit for bit, and leave
    every mask byte, slot word, list count, sparse gradient row and the item
    side table zero after each step."""
    e, g = _graph()
    kw = dict(cred=synthetic_credibility(3000, 5), emb_dim=dim, num_layers=K, batch_size=256,
              frontier=True, fuse_adam=fuse, seed=11)
    a = FusedTrainer(g, "v2_pop", **kw)
    monkeypatch.setenv("BBGR_BATCH_FUSED", "0")
    b = FusedTrainer(g, "v2_pop", **kw)
    assert a.batch_fused and not b.batch_fused
    for _ in range(4):
        assert float(a.step()) == float(b.step())
        assert not a._fused_pending
        for t in (a.mask_u, a.mask_i, a.g_uf, a.g_if, a.item_count):
            assert int(t.abs().sum()) == 0
        if a.slot_bits is not None:
            assert int(a.slot_bits.abs().sum()) == 0
        side = getattr(a, "_g_item_side", None)
        if side is not None:
            assert float(side.abs().sum()) == 0.0
    _assert_same(a, b)
    # caller batches (repeated users) take the same launches
    users = torch.tensor([5, 5, 17, 2999, 0, 17], dtype=torch.int64)
    assert float(a.step(users)) == float(b.step(users))
    _assert_same(a, b)
    assert int(a.mask_i.abs().sum()) == 0 and int(a.item_count.abs().sum()) == 0


def test_fused_batch_bookkeeping_graph_replay():
    """A captured step with the fused bookkeeping replays bitwise the eager
    steps (the list count is restored on the device inside the graph)."""
    e, g = _graph()
    kw = dict(cred=synthetic_credibility(3000, 5), emb_dim=64, num_layers=3, batch_size=256,
              frontier=True, fuse_adam=True, seed=13)
    a, b = FusedTrainer(g, "v2_pop", **kw), FusedTrainer(g, "v2_pop", **kw)
    assert a.batch_fused
    gs = GraphedStep(a)   # (a trainer that has not stepped takes its first step eagerly)
    assert float(gs.first_loss) == float(b.step())
    for _ in range(5):
        assert float(gs.step()) == float(b.step())
    _assert_same(a, b)
    assert int(a.item_count.abs().sum()) == 0 and int(a.mask_i.abs().sum()) == 0


@pytest.mark.parametrize("variant,fuse,K", [("v2_pop", True, 3), ("v2_pop", False, 3),
                                            ("v2_pop", True, 2), ("v2_pop", True, 1),
                                            ("cu_fair", True, 3), ("cu_fair", False, 2)])
def test_packed_item_mask_step_is_bitwise_the_byte_mask_step(variant, fuse, K, monkeypatch):
    """Frontier (GS and Jacobi): the first backward user product tests its
    edges on the item mask packed one bit per item (bbgr_mask_pack +
    src_mask_bits) — losses, weights and moments equal the byte-mask step's
    bit for bit (BBGR_MASK_BITS=0), through graph capture too."""
    e, g = _graph()
    kw = dict(cred=synthetic_credibility(3000, 5), emb_dim=64, num_layers=K, batch_size=256,
              frontier=True, fuse_adam=fuse, seed=17)
    a = FusedTrainer(g, variant, **kw)
    monkeypatch.setenv("BBGR_MASK_BITS", "0")
    b = FusedTrainer(g, variant, **kw)
    assert a.mask_i_bits is not None and b.mask_i_bits is None
    for _ in range(4):
        assert float(a.step()) == float(b.step())
    _assert_same(a, b)
    if K >= 2:
        gs = GraphedStep(a)
        for _ in range(3):
            assert float(gs.step()) == float(b.step())
        _assert_same(a, b)


def test_batch_begin_end_kernels_direct():
    """bbgr_batch_begin / bbgr_batch_end through the C ABI: the masks, the
    frontier list (each flagged item once), the slot bits and the sparse
    gradient rows' reset, with repeated users, ids outside the tables
    (skipped: -1, U, I) and an empty batch; everything zero again after."""
    from bbgr import _lib
    from bbgr._lib import ptr
    e, g = _graph()
    U, I, d = g.num_users, g.num_items, 64
    uc = g.user_csr
    slot_map = g.user_item_slots()
    users = torch.tensor([5, 5, 17, -1, U, 0, 2999, 17], dtype=torch.int64, device=DEV)
    pos = torch.tensor([1, 1, 3, 4, 5, I, -1, 7], dtype=torch.int64, device=DEV)
    neg = torch.tensor([2, 9, 3, 4, 6, 8, 1199, -1], dtype=torch.int64, device=DEV)
    B = users.numel()
    posneg = torch.cat([pos, neg])
    mask_u = _lib.byte_mask(U, DEV)
    mask_i = _lib.byte_mask(I, DEV)
    lst = torch.full((I,), -7, dtype=torch.int64, device=DEV)
    cnt = torch.zeros(1, dtype=torch.int64, device=DEV)
    bits = torch.zeros(uc.nnz // 32 + 4, dtype=torch.int32, device=DEV)
    gu = torch.zeros(U, d, device=DEV)
    gi = torch.zeros(I, d, device=DEV)
    gs = torch.zeros(I, d, device=DEV)
    a = _lib.BatchArgs()
    a.batch, a.users, a.pos, a.neg = B, ptr(users), ptr(posneg), ptr(posneg) + 8 * B
    a.n_users, a.n_items = U, I
    a.user_indptr, a.user_indices = ptr(uc.indptr), ptr(uc.indices)
    a.mask_u, a.mask_i, a.list, a.count = ptr(mask_u), ptr(mask_i), ptr(lst), ptr(cnt)
    a.slot_map, a.slot_bits = ptr(slot_map), ptr(bits)
    a.g_u, a.g_i, a.g_side = ptr(gu), ptr(gi), ptr(gs)
    a.ld_gu = a.ld_gi = a.ld_side = d
    a.d = d
    _lib.call("bbgr_batch_begin", ctypes.byref(a), _lib.stream_handle())
    torch.cuda.synchronize()
    ok_u = users[(users >= 0) & (users < U)]
    want_u = torch.zeros(U, dtype=torch.uint8, device=DEV)
    want_u[ok_u] = 1
    assert torch.equal(mask_u[:U], want_u)
    ip = uc.indptr.long()
    want_i = torch.zeros(I, dtype=torch.uint8, device=DEV)
    items = posneg[(posneg >= 0) & (posneg < I)]
    want_i[items] = 1
    slots = []
    for u in ok_u.unique().tolist():
        cols = uc.indices[ip[u]: ip[u + 1]].long()
        want_i[cols] = 1
        slots.append(slot_map[ip[u]: ip[u + 1]].long())
    assert torch.equal(mask_i[:I], want_i)
    n = int(cnt.item())
    listed = lst[:n]
    assert n == int(want_i.sum()) and listed.unique().numel() == n
    assert bool((want_i[listed] == 1).all())
    want_bits = torch.zeros(bits.numel() * 32, dtype=torch.bool, device=DEV)
    want_bits[torch.cat(slots)] = True
    got_bits = ((bits.view(-1, 1).long() & 0xFFFFFFFF) >> torch.arange(32, device=DEV)) & 1
    assert torch.equal(got_bits.view(-1).bool(), want_bits)
    # the step's sparse gradient rows, then the end restores every table
    gu[ok_u] = 1.0
    gi[items] = 2.0
    gs[items] = 3.0
    _lib.call("bbgr_batch_end", ctypes.byref(a), _lib.stream_handle())
    torch.cuda.synchronize()
    for t in (mask_u, mask_i, bits, cnt, gu, gi, gs):
        assert float(t.abs().sum()) == 0.0
    # an empty batch: no launch but the count reset
    cnt.fill_(5)
    a.batch = 0
    _lib.call("bbgr_batch_begin", ctypes.byref(a), _lib.stream_handle())
    _lib.call("bbgr_batch_end", ctypes.byref(a), _lib.stream_handle())
    torch.cuda.synchronize()
    assert int(cnt.item()) == 0 and float(mask_i.abs().sum()) == 0.0


@pytest.mark.parametrize("ranked", [False, True])
def test_rows_mark_is_the_separate_marking(ranked):
    """bbgr_rows_mark (propagate_rows' marking in one launch) against its
    definition by the separate marking launches: the graph-order masks, the
    caller-order masks, the distinct-user list and the item frontier list (as
    sets; each listed once, counts equal), with repeated ids, ids outside the
    tables (-1, U, I, skipped), caller ids mapped through rank tables or not,
    and more items than users and the reverse."""
    from bbgr import _lib
    from bbgr._lib import ptr
    e, g = _graph()
    U, I = g.num_users, g.num_items
    uc = g.user_csr
    gen = torch.Generator().manual_seed(11 + ranked)
    urank = torch.randperm(U, generator=gen).to(DEV) if ranked else None
    irank = torch.randperm(I, generator=gen).to(DEV) if ranked else None
    for nu, ni in ((9, 18), (40, 3), (0, 5), (6, 0)):
        users = torch.randint(0, U, (nu,), generator=gen).to(DEV)
        items = torch.randint(0, I, (ni,), generator=gen).to(DEV)
        if nu >= 3:
            users[0], users[1], users[2] = -1, U, users[3 % nu]
        if ni >= 3:
            items[0], items[1], items[2] = I, -1, items[-1]

        def run(fused):
            m = {k: _lib.byte_mask(n, DEV) for k, n in
                 (("mu", U), ("mi", I), ("fr", I), ("mu_in", U), ("mi_in", I))}
            ul = torch.full((max(nu, 1),), -7, dtype=torch.int64, device=DEV)
            fl = torch.full((I,), -7, dtype=torch.int64, device=DEV)
            cnt = torch.zeros(2, dtype=torch.int64, device=DEV)
            st = _lib.stream_handle()
            if fused:
                a = _lib.RowsMarkArgs()
                a.n_users_listed, a.n_items_listed = nu, ni
                a.users, a.items = ptr(users), ptr(items)
                a.n_users, a.n_items = U, I
                a.user_rank = ptr(urank) if ranked else None
                a.item_rank = ptr(irank) if ranked else None
                a.user_indptr, a.user_indices = ptr(uc.indptr), ptr(uc.indices)
                a.mask_u, a.mask_i, a.frontier = ptr(m["mu"]), ptr(m["mi"]), ptr(m["fr"])
                a.mask_u_in, a.mask_i_in = ptr(m["mu_in"]), ptr(m["mi_in"])
                a.user_list, a.user_count = ptr(ul), ptr(cnt)
                a.frontier_list, a.frontier_count = ptr(fl), ptr(cnt) + 8
                _lib.call("bbgr_rows_mark", ctypes.byref(a), st)
            else:
                def rows(ids, n, rank):
                    ok = (ids >= 0) & (ids < n)
                    r = torch.full_like(ids, -1)
                    r[ok] = rank[ids[ok]] if rank is not None else ids[ok]
                    return r
                ui, ii = rows(users, U, urank), rows(items, I, irank)
                L = lambda *x: _lib.call("bbgr_mark_list", *x, st)
                R = lambda *x: _lib.call("bbgr_mark_rows", *x, st)
                L(nu, ptr(ui), None, None, ptr(m["mu"]), U, ptr(ul), ptr(cnt))
                R(ni, ptr(ii), 1, ptr(m["mi"]), I)
                L(ni, ptr(ii), None, None, ptr(m["fr"]), I, ptr(fl), ptr(cnt) + 8)
                L(nu, ptr(ui), ptr(uc.indptr), ptr(uc.indices), ptr(m["fr"]), I, ptr(fl),
                  ptr(cnt) + 8)
                R(nu, ptr(users), 1, ptr(m["mu_in"]), U)
                R(ni, ptr(items), 1, ptr(m["mi_in"]), I)
            torch.cuda.synchronize()
            c = cnt.tolist()
            return m, ul[:c[0]].sort().values, fl[:c[1]].sort().values

        mf, ulf, flf = run(True)
        ms, uls, fls = run(False)
        for k in mf:
            assert torch.equal(mf[k], ms[k]), (k, nu, ni)
        assert torch.equal(ulf, uls) and torch.equal(flf, fls), (nu, ni)
        assert ulf.unique().numel() == ulf.numel() and flf.unique().numel() == flf.numel()
        assert int(mf["fr"][:I].sum()) == flf.numel() and int(mf["mu"][:U].sum()) == ulf.numel()
