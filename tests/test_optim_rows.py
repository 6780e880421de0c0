"""CPU: FusedAdam's graph-order moments (optim.FusedAdam._graph_rows).

The in-backward step (bbgr::bpr_adam_backward, ABI 9 adam_moments_unmapped)
keeps a degree-ordered drop-in pair's moments in the graph's row order; the
optimizer converts them there once and back wherever they leave it. The
conversions are plain torch index ops, checked here without a GPU: a graph
row r holds the caller row map[r]; state_dict() and moments() give the
caller's order without disturbing the internal tables; a second map
converts through the caller's order; load_state_dict() restarts in the
caller's order, as torch.optim.Adam's state does.
"""
import copy

import torch

from bbgr.optim import FusedAdam


def _opt(rows=7, d=3):
    torch.manual_seed(0)
    p = torch.nn.Parameter(torch.randn(rows, d))
    q = torch.nn.Parameter(torch.randn(2, d))
    o = FusedAdam([p, q], lr=1e-3, fuse_backward=True)
    for t in (p, q):
        st = o._init_state(t)
        st["exp_avg"].copy_(torch.randn(t.shape))
        st["exp_avg_sq"].copy_(torch.rand(t.shape))
        st["step"] += 3
    return o, p, q


def test_graph_rows_round_trip_and_caller_order_views():
    o, p, q = _opt()
    m0, v0 = (t.clone() for t in o.moments(p))
    sd0 = copy.deepcopy(o.state_dict())   # (torch's state_dict shares the live dicts)
    perm = torch.randperm(p.shape[0])            # map[graph row] = caller row
    o._to_graph_rows(p, perm)
    st = o.state[p]
    assert torch.equal(st["exp_avg"], m0[perm]) and torch.equal(st["exp_avg_sq"], v0[perm])
    o._to_graph_rows(p, perm)                    # the same map again: nothing moves
    assert torch.equal(st["exp_avg"], m0[perm])
    m, v = o.moments(p)
    assert torch.equal(m, m0) and torch.equal(v, v0)
    assert torch.equal(st["exp_avg"], m0[perm])  # moments() copied, did not convert
    sd = o.state_dict()
    for k in sd0["state"]:
        for key in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(sd["state"][k][key], sd0["state"][k][key]), (k, key)
    assert torch.equal(st["exp_avg"], m0[perm])  # state_dict() neither
    other = torch.randperm(p.shape[0])           # another pair's order
    o._to_graph_rows(p, other)
    assert torch.equal(o.state[p]["exp_avg"], m0[other])
    o._to_caller_rows(p)
    assert torch.equal(o.state[p]["exp_avg"], m0) and torch.equal(o.state[p]["exp_avg_sq"], v0)
    assert not o._graph_rows


def test_load_state_dict_restarts_in_the_callers_order():
    o, p, q = _opt()
    m0 = o.moments(p)[0].clone()
    o._to_graph_rows(p, torch.randperm(p.shape[0]))
    sd = copy.deepcopy(o.state_dict())
    o2, p2, q2 = _opt()
    o2._to_graph_rows(p2, torch.randperm(p2.shape[0]))
    o2.load_state_dict(sd)
    assert not o2._graph_rows
    assert torch.equal(o2.state[p2]["exp_avg"], m0)
    assert int(o2.state[p2]["step"]) == 3
