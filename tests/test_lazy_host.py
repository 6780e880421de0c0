"""CPU: the host mechanics of the drop-in's deferred final tables (bbgr.lazy).

The device path (bbgr::propagate_rows, bitwise the dense step) is tested in
tests/test_gpu_lazy.py; here the DeferredFinal tensor itself runs on CPU
tables with stand-in compute functions: metadata without compute, compute
once on first use, autograd through the computed tables, the weight-version
guard, and bpr_loss's batch-rows dispatch.
"""
import pytest
import torch

from bbgr import lazy


def _pair(calls, U=6, I=4, d=3):
    torch.manual_seed(0)
    u0 = torch.randn(U, d, requires_grad=True)
    i0 = torch.randn(I, d, requires_grad=True)

    def full():
        calls.append("full")
        return u0 * 2.0, i0 * 3.0

    def rows(users, items):
        calls.append(("rows", users.tolist(), items.tolist()))
        return u0 * 2.0, i0 * 3.0

    p = lazy._Pending(full, rows, u0, i0)
    a = lazy.DeferredFinal(p, 0, torch.empty(U, d), True)
    b = lazy.DeferredFinal(p, 1, torch.empty(I, d), True)
    return u0, i0, a, b


def test_metadata_answers_without_compute():
    calls = []
    u0, i0, a, b = _pair(calls)
    assert a.shape == (6, 3) and b.size(0) == 4 and a.dim() == 2 and len(b) == 4
    assert a.dtype == torch.float32 and a.device.type == "cpu" and a.requires_grad
    assert a.numel() == 18
    assert calls == []


def test_first_use_computes_once_and_results_are_plain_tensors():
    calls = []
    u0, i0, a, b = _pair(calls)
    x = a[1]
    assert type(x) is torch.Tensor and calls == ["full"]
    assert torch.equal(x, (u0 * 2.0)[1])
    y = b + 1
    assert type(y) is torch.Tensor and calls == ["full"]      # cached
    assert torch.equal(y, i0 * 3.0 + 1)
    assert "tensor(" in repr(a)
    (a.sum() + b.sum()).backward()                            # the computed graph
    assert torch.equal(u0.grad, torch.full_like(u0, 2.0))
    assert torch.equal(i0.grad, torch.full_like(i0, 3.0))


def test_use_after_in_place_weight_update_raises():
    calls = []
    u0, i0, a, b = _pair(calls)
    with torch.no_grad():
        u0.add_(1.0)
    with pytest.raises(RuntimeError, match="weights changed"):
        a * 2
    with pytest.raises(RuntimeError, match="weights changed"):
        lazy.batch_finals(a, b, [0], [1], [2])


def test_batch_finals_takes_the_rows_path_for_one_calls_pair_only():
    calls = []
    u0, i0, a, b = _pair(calls)
    uf, itf, users, pos, neg = lazy.batch_finals(a, b, [0, 2], [1, 3], [0, 0])
    assert calls == [("rows", [0, 2], [1, 3, 0, 0])]
    assert users.dtype == torch.int64 and type(uf) is torch.Tensor
    # tables of two different calls, or a swapped pair: the whole tables
    calls2 = []
    _, _, a2, b2 = _pair(calls2)
    uf, itf, *_ = lazy.batch_finals(a, b2, [0], [1], [2])
    assert "full" in calls and "full" in calls2
    # a plain tensor passes through
    t = torch.zeros(2, 3)
    assert lazy.batch_finals(t, t, [0], [0], [0])[0] is t


def test_not_supported_on_cpu_tables():
    assert not lazy.supported(torch.zeros(2, 2), torch.zeros(2, 2))
