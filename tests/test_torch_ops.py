"""CPU: the C++ operator library (csrc/torch_ops.cpp -> libbbgr_torch.so).

No kernels run here: the checks use the Meta kernels (what torch.compile
traces), the Autograd kernels on meta tensors, TorchScript resolution (a
libtorch / TorchScript caller reaches the same operators), and the schemas
bbgr/ops.py documents. The HIP kernels are checked on the GPU
(tests/test_gpu_ops.py: bitwise against the Python chain, compile, capture).
"""
import pytest
import torch

from bbgr import ops

SCHEMAS = {
    "propagate": "bbgr::propagate(Tensor u0, Tensor i0, int pair_key, int num_layers, str order)"
                 " -> (Tensor, Tensor)",
    "propagate_backward_rows": "bbgr::propagate_backward_rows(Tensor iu, Tensor vu, Tensor gI, "
                               "int num_users, int pair_key, int num_layers, str order, "
                               "Tensor? ii=None, Tensor? vi=None) -> (Tensor, Tensor)",
    "bpr_loss": "bbgr::bpr_loss(Tensor uf, Tensor itf, Tensor ue, Tensor ie, Tensor users, "
                "Tensor pos, Tensor neg, float reg, Tensor? pop, float lambda_fair) -> Tensor",
}
NAMES = ["propagate", "propagate_backward", "propagate_backward_rows", "jacobi_layer",
         "jacobi_layer_backward", "propagate_sym", "propagate_sym_backward", "bpr_loss",
         "bpr_loss_backward", "bpr_loss_sparse_ego", "_register_pair", "_unregister_pair",
         "_counters", "_item_table_sets"]


def test_every_operator_is_registered_from_cpp():
    for n in NAMES:
        op = getattr(torch.ops.bbgr, n).default
        assert op._schema.name == f"bbgr::{n}"
    for n, s in SCHEMAS.items():
        assert str(getattr(torch.ops.bbgr, n).default._schema) == s
    for n in ("propagate", "jacobi_layer", "propagate_sym", "bpr_loss", "bpr_loss_sparse_ego"):
        for key in ("CUDA", "Meta", "Autograd"):
            assert torch._C._dispatch_has_kernel_for_dispatch_key(f"bbgr::{n}", key), (n, key)
    for n in ("propagate_backward", "propagate_backward_rows", "bpr_loss_backward"):
        assert torch._C._dispatch_has_kernel_for_dispatch_key(f"bbgr::{n}", "CUDA")
        assert not torch._C._dispatch_has_kernel_for_dispatch_key(f"bbgr::{n}", "Autograd")


def test_no_python_operator_definitions():
    """The package defines no torch.library operators in Python (ops.py only
    loads the library and registers operator pairs)."""
    import inspect
    src = inspect.getsource(ops)
    assert "custom_op" not in src and "register_fake" not in src
    assert ops.propagate is torch.ops.bbgr.propagate


@pytest.mark.parametrize("order", ["gs", "jacobi"])
def test_meta_autograd_shapes(order):
    u = torch.empty(10, 8, device="meta", requires_grad=True)
    i = torch.empty(5, 8, device="meta", requires_grad=True)
    uf, itf = torch.ops.bbgr.propagate(u, i, 1, 3, order)
    assert uf.shape == u.shape and itf.shape == i.shape
    assert uf.grad_fn.name() == ops.PROPAGATE_NODE
    (uf.sum() + itf.sum()).backward()
    assert u.grad.shape == u.shape and i.grad.shape == i.shape
    x = torch.empty(15, 8, device="meta", requires_grad=True)
    torch.ops.bbgr.propagate_sym(x, 1, 2).sum().backward()
    assert x.grad.shape == x.shape
    a, b = torch.ops.bbgr.jacobi_layer(u, i, 1)
    assert a.shape == i.shape and b.shape == u.shape
    users = torch.zeros(4, dtype=torch.long, device="meta")
    loss = torch.ops.bbgr.bpr_loss(uf, itf, u, i, users, users, users, 1e-4, None, 0.0)
    assert loss.shape == () and "Bpr" in loss.grad_fn.name()


def test_torchscript_resolves_the_operators():
    """TorchScript (and through it a libtorch caller) binds torch.ops.bbgr.*."""
    @torch.jit.script
    def step(u0: torch.Tensor, i0: torch.Tensor, key: int):
        uf, itf = torch.ops.bbgr.propagate(u0, i0, key, 3, "gs")
        return (uf * itf[:1]).sum()

    assert "bbgr::propagate" in str(step.graph)
    out = step(torch.empty(6, 4, device="meta"), torch.empty(3, 4, device="meta"), 7)
    assert out.shape == ()


def test_cpu_tensors_fail_loudly():
    """No CPU kernel exists (no fallback): CPU tensors raise."""
    torch.ops.bbgr._unregister_pair(10**9)      # an unknown key: a no-op
    with pytest.raises(NotImplementedError, match="CPU"):
        torch.ops.bbgr.propagate(torch.zeros(3, 4), torch.zeros(2, 4), 1, 1, "gs")
