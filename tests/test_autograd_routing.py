"""CPU: when bpr.bpr_loss may hand the ego-L2 gradient back as sparse rows.

bpr._receives_dense_grad decides from the autograd graph alone (no kernels),
so it is checked here on CPU with a stand-in two-output op shaped like
bbgr::propagate (registered as a propagate node for these tests): the sparse
form is chosen only when the final tables come straight out of that node and
it also returns a dense gradient for the same leaf weights, never for
detached / derived tables, other nodes with a direct edge to the weight
(ADVICE r2), under no_grad, or while dynamo compiles."""
import pytest
import torch
from torch.library import custom_op

from bbgr import bpr


@custom_op("bbgr_test::two_tables", mutates_args=())
def two_tables(u0: torch.Tensor, i0: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    return u0 * 2, i0 * 3


@two_tables.register_fake
def _(u0, i0):
    return u0.new_empty(u0.shape), i0.new_empty(i0.shape)


two_tables.register_autograd(lambda ctx, gu, gi: (gu * 2, gi * 3),
                             setup_context=lambda ctx, inputs, output: None)


@pytest.fixture(autouse=True)
def _stand_in_is_a_propagate_node(monkeypatch):
    monkeypatch.setattr(bpr, "PROPAGATE_NODES", bpr.PROPAGATE_NODES |
                        {"GeneratedBackwardFor_bbgr_test_two_tables_defaultBackward"})


def _weights():
    return torch.nn.Embedding(6, 4).weight, torch.nn.Embedding(5, 4).weight


def test_dense_node_outputs_take_the_sparse_form():
    wu, wi = _weights()
    uf, itf = two_tables(wu, wi)
    assert bpr._receives_dense_grad(uf, wu) and bpr._receives_dense_grad(itf, wi)


def test_other_tables_keep_the_dense_form():
    wu, wi = _weights()
    uf, itf = two_tables(wu, wi)
    assert not bpr._receives_dense_grad(uf.detach(), wu)      # no graph
    assert not bpr._receives_dense_grad(uf * 1.0, wu)         # a derived table
    assert not bpr._receives_dense_grad(wu + uf.detach(), wu)  # Add with a leaf edge
    other, _ = _weights()
    assert not bpr._receives_dense_grad(two_tables(other, wi)[0], wu)
    with torch.no_grad():
        assert not bpr._receives_dense_grad(uf, wu)
    frozen = wu.detach()
    assert not bpr._receives_dense_grad(two_tables(frozen, wi)[0], frozen)


def test_not_while_compiling():
    wu, wi = _weights()
    uf, _ = two_tables(wu, wi)
    seen = []

    def probe(x):
        seen.append(bpr._receives_dense_grad(uf, wu))
        return x + 1

    torch.compile(probe, backend="eager")(torch.ones(2))
    assert seen and not any(seen)


@pytest.mark.parametrize("n,hi", [(1, 5), (2, 1), (7, 3), (1000, 50), (16384, 1_000_000)])
def test_first_slot_is_the_first_occurrence(n, hi):
    """bpr._first_slot (the ego rows' slot of each triple, by a sort +
    lower-bound search; the C++ operators use bbgr_first_slot, an atomic
    minimum per row, checked against this in tests/test_gpu_parity.py): slot[b]
    is the smallest b' with ids[b'] == ids[b]."""
    g = torch.Generator().manual_seed(n + hi)
    ids = torch.randint(0, hi, (n,), generator=g)
    first = {}
    for b, v in enumerate(ids.tolist()):
        first.setdefault(v, b)
    want = torch.tensor([first[v] for v in ids.tolist()])
    assert torch.equal(bpr._first_slot(ids), want)
