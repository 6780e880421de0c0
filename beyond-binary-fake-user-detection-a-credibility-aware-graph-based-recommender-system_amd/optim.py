"""FusedAdam: torch.optim.Adam semantics on the bbgr_adam HIP kernel.

Drop-in for ``torch.optim.Adam(model.parameters(), lr=cfg.lr)``
(Version-2/lighgcn_cu_pop.py:793, step at :863): same defaults
(betas=(0.9, 0.999), eps=1e-8, weight_decay=0), same state keys
(``step``, ``exp_avg``, ``exp_avg_sq``) so state_dicts interchange.
Bias corrections are computed on the host in double, as torch does.
"""
from __future__ import annotations

import math

import torch

from . import _lib
from ._lib import call, ptr, stream_handle


class AdamRows:
    """Arguments of a fused Adam step applied inside an SpMM epilogue
    (bbgr_spmm_args.adam_*): the row gradient never touches HBM."""

    def __init__(self, param, exp_avg, exp_avg_sq, step: int, lr: float, beta1: float = 0.9,
                 beta2: float = 0.999, eps: float = 1e-8, weight_decay: float = 0.0):
        self.param, self.exp_avg, self.exp_avg_sq = param, exp_avg, exp_avg_sq
        self.lr, self.beta1, self.beta2, self.eps, self.wd = lr, beta1, beta2, eps, weight_decay
        self.bc1 = 1.0 - beta1 ** step
        self.bc2s = math.sqrt(1.0 - beta2 ** step)

    def apply(self, grad: torch.Tensor) -> None:
        """The same step, unfused (bbgr_adam on a materialised gradient)."""
        call("bbgr_adam", self.param.numel(), ptr(self.param), ptr(grad), ptr(self.exp_avg),
             ptr(self.exp_avg_sq), float(self.lr), float(self.beta1), float(self.beta2),
             float(self.eps), float(self.wd), 1.0, float(self.bc1), float(self.bc2s),
             stream_handle())

    def fill(self, a) -> None:
        from ._lib import ld
        a.adam_param, a.adam_exp_avg = ptr(self.param), ptr(self.exp_avg)
        a.adam_exp_avg_sq, a.adam_ld = ptr(self.exp_avg_sq), ld(self.param)
        a.adam_lr, a.adam_beta1, a.adam_beta2 = self.lr, self.beta1, self.beta2
        a.adam_eps, a.adam_weight_decay = self.eps, self.wd
        a.adam_bias_correction1, a.adam_bias_correction2_sqrt = self.bc1, self.bc2s


def adam_step(param: torch.Tensor, grad: torch.Tensor, exp_avg: torch.Tensor,
              exp_avg_sq: torch.Tensor, step: int, lr: float, beta1: float = 0.9,
              beta2: float = 0.999, eps: float = 1e-8, weight_decay: float = 0.0,
              grad_scale: float = 1.0) -> None:
    for t in (param, grad, exp_avg, exp_avg_sq):
        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
            raise ValueError("adam_step takes contiguous fp32 device tensors")
        if t.numel() != param.numel():
            raise ValueError("adam_step: size mismatch")
    bc1 = 1.0 - beta1 ** step
    bc2s = math.sqrt(1.0 - beta2 ** step)
    call("bbgr_adam", param.numel(), ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq),
         float(lr), float(beta1), float(beta2), float(eps), float(weight_decay),
         float(grad_scale), float(bc1), float(bc2s), stream_handle())


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0):
        if lr < 0.0 or eps < 0.0 or not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError("invalid Adam hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                _lib.require_gpu(p)
                st = self.state[p]
                if not st:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                adam_step(p.data, p.grad.contiguous(), st["exp_avg"], st["exp_avg_sq"],
                          int(st["step"].item()), group["lr"], b1, b2, group["eps"],
                          group["weight_decay"])
        return loss
