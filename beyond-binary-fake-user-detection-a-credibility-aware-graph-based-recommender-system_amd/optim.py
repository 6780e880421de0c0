"""FusedAdam: torch.optim.Adam semantics on the bbgr_adam HIP kernel.

Drop-in for ``torch.optim.Adam(model.parameters(), lr=cfg.lr)``
(Version-2/lighgcn_cu_pop.py:793, step at :863): same defaults
(betas=(0.9, 0.999), eps=1e-8, weight_decay=0), same state keys
(``step``, ``exp_avg``, ``exp_avg_sq``) so state_dicts interchange.
Bias corrections are computed on the host in double, as torch does.
"""
from __future__ import annotations

import math
import warnings

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_handle


def bias_corrections(n: int, beta1: float = 0.9, beta2: float = 0.999) -> np.ndarray:
    """float32 [n, 2]: (1 - beta1^t, sqrt(1 - beta2^t)) for t = 1..n, with the
    host path's arithmetic (libm pow and sqrt in double, then rounded to float
    as the ctypes float argument rounds it)."""
    t = np.arange(1, n + 1, dtype=np.float64)
    bc = np.empty((n, 2), dtype=np.float64)
    bc[:, 0] = 1.0 - np.power(np.float64(beta1), t)
    bc[:, 1] = np.sqrt(1.0 - np.power(np.float64(beta2), t))
    return bc.astype(np.float32)


def exact_table_steps(beta1: float = 0.9, beta2: float = 0.999) -> int:
    """A bias-correction table length past whose end every step's fp32
    constants are exactly (1.0f, 1.0f): beta^t < 2^-25 for both betas makes
    1 - beta1^t and sqrt(1 - beta2^t) round to 1.0f (0.9 / 0.999: ~17k steps).
    The kernels clamp t to the table's end, so a table at least this long
    holds every step's constants (tests/test_oracle.py checks it)."""
    n = 1
    for b in (beta1, beta2):
        if 0.0 < b < 1.0:
            n = max(n, int(math.ceil(-25.0 * math.log(2.0) / math.log(b))) + 1)
    return n


class DeviceStepState:
    """Device-resident step scalars of a graph-captured training step
    (include/bbgr.h, bbgr_step_begin): state = int64 {t, counter, next counter,
    table length} and the bias-correction table bc[t-1] = (1 - beta1^t,
    sqrt(1 - beta2^t)), computed here in double exactly as the host path does
    (then float). The kernels clamp t to the table (exact past its end)."""

    def __init__(self, device, step: int, counter: int, max_steps: int = 1 << 20,
                 beta1: float = 0.9, beta2: float = 0.999):
        # at least exact_table_steps() entries, so the kernels' clamp of t to
        # the table end is exact (every later step's corrections round to 1.0f)
        self.max_steps = max(int(max_steps), exact_table_steps(beta1, beta2))
        self.beta1, self.beta2 = beta1, beta2
        self.state = torch.tensor([step, counter - 1, counter, self.max_steps],
                                  dtype=torch.int64, device=device)
        self.bc_table = torch.from_numpy(bias_corrections(self.max_steps, beta1, beta2)).to(device)

    def begin(self) -> None:
        """t += 1; this step's sampler counter = next; next += 1 (on the device)."""
        call("bbgr_step_begin", ptr(self.state), stream_handle())


class AdamRows:
    """Arguments of a fused Adam step applied inside an SpMM epilogue
    (bbgr_spmm_args.adam_*): the row gradient never touches HBM. With
    `dev` (DeviceStepState) the step t and bias corrections are read on the
    device (graph-captured steps). `grad` (a table like param): the gradient
    is grad_scale * grad[row] instead of the launch's row value, which is then
    still written to y (bbgr_spmm_args.adam_grad): another table's Adam riding
    on a product over the same rows."""

    def __init__(self, param, exp_avg, exp_avg_sq, step: int, lr: float, beta1: float = 0.9,
                 beta2: float = 0.999, eps: float = 1e-8, weight_decay: float = 0.0,
                 dev: DeviceStepState | None = None, grad=None, grad_scale: float = 1.0):
        self.param, self.exp_avg, self.exp_avg_sq = param, exp_avg, exp_avg_sq
        if grad is not None and (grad.shape != param.shape or grad.dtype != param.dtype):
            raise ValueError("AdamRows: grad must be a table shaped like param")
        self.grad, self.grad_scale = grad, grad_scale
        self.lr, self.beta1, self.beta2, self.eps, self.wd = lr, beta1, beta2, eps, weight_decay
        self.bc1 = 1.0 - beta1 ** step
        self.bc2s = math.sqrt(1.0 - beta2 ** step)
        self.dev = dev

    def apply(self, grad: torch.Tensor) -> None:
        """The same step, unfused (bbgr_adam on a materialised gradient)."""
        adam_step(self.param, grad, self.exp_avg, self.exp_avg_sq, 0, self.lr, self.beta1,
                  self.beta2, self.eps, self.wd, dev=self.dev,
                  bc=(self.bc1, self.bc2s))

    def fill(self, a) -> None:
        from ._lib import ld
        a.adam_param, a.adam_exp_avg = ptr(self.param), ptr(self.exp_avg)
        a.adam_exp_avg_sq, a.adam_ld = ptr(self.exp_avg_sq), ld(self.param)
        a.adam_lr, a.adam_beta1, a.adam_beta2 = self.lr, self.beta1, self.beta2
        a.adam_eps, a.adam_weight_decay = self.eps, self.wd
        a.adam_bias_correction1, a.adam_bias_correction2_sqrt = self.bc1, self.bc2s
        if self.dev is not None:
            a.adam_bc_table, a.adam_state = ptr(self.dev.bc_table), ptr(self.dev.state)
        if self.grad is not None:
            a.adam_grad, a.adam_grad_ld = ptr(self.grad), ld(self.grad)
            a.adam_grad_scale = self.grad_scale


def adam_step(param: torch.Tensor, grad: torch.Tensor, exp_avg: torch.Tensor,
              exp_avg_sq: torch.Tensor, step: int, lr: float, beta1: float = 0.9,
              beta2: float = 0.999, eps: float = 1e-8, weight_decay: float = 0.0,
              grad_scale: float = 1.0, dev: DeviceStepState | None = None,
              bc: tuple | None = None) -> None:
    """torch.optim.Adam's step `step` on one tensor (bbgr_adam); with `dev`
    the step and bias corrections come from the device step state instead
    (bbgr_adam_dev; `step` is then ignored)."""
    for t in (param, grad, exp_avg, exp_avg_sq):
        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
            raise ValueError("adam_step takes contiguous fp32 device tensors")
        if t.numel() != param.numel():
            raise ValueError("adam_step: size mismatch")
    if dev is not None:
        call("bbgr_adam_dev", param.numel(), ptr(param), ptr(grad), ptr(exp_avg),
             ptr(exp_avg_sq), float(lr), float(beta1), float(beta2), float(eps),
             float(weight_decay), float(grad_scale), ptr(dev.bc_table), ptr(dev.state),
             stream_handle())
        return
    bc1, bc2s = bc if bc is not None else (1.0 - beta1 ** step, math.sqrt(1.0 - beta2 ** step))
    call("bbgr_adam", param.numel(), ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq),
         float(lr), float(beta1), float(beta2), float(eps), float(weight_decay),
         float(grad_scale), float(bc1), float(bc2s), stream_handle())


# parameters owned by a FusedAdam in backward mode: id -> (weakref(param), weakref(opt))
_IN_BACKWARD: dict = {}


def backward_optimizer(*params):
    """The FusedAdam(fuse_backward=True) that owns every one of `params` in one
    param group, or None."""
    found = None
    for p in params:
        e = _IN_BACKWARD.get(id(p))
        if e is None or e[0]() is not p:
            return None
        o = e[1]()
        if o is None or (found is not None and o is not found):
            return None
        found = o
    if found is None or found._group_of(params) is None:
        return None
    return found


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam on the bbgr_adam kernel (module docstring).

    fuse_backward=True (the drop-in LightGCN of Version-2 / Method A, GS
    order, num_layers >= 2): the step of the model's two embedding tables runs
    INSIDE loss.backward(), in the epilogues of the last backward SpMMs
    (bbgr::bpr_adam_backward): the user step on the last user product, the item
    step on the last item product, so neither gradient table is written nor
    re-read. Those parameters then get no .grad, and the following step()
    leaves them alone (they were stepped already); anything else in the
    optimizer steps as usual. The reference's loop (zero_grad, backward,
    step: Version-2/lighgcn_cu_pop.py:861-863) runs unchanged. Each backward
    through bpr_loss is one optimizer step. The update equals the separate
    step's up to rounding: the ego-L2 rows join the gradient before the last
    products' epilogues, not after them (FusedTrainer's order).

    On a degree-ordered drop-in graph (the default) the in-backward step keeps
    those two tables' exp_avg / exp_avg_sq in the graph's row order, so the
    fused epilogue streams them and reads only the weight rows through the row
    map. The optimizer converts them once, and back wherever they leave it:
    state_dict(), moments(), and a step() that updates them outside the
    backward. load_state_dict() takes the caller's order, as torch's Adam.
    With use_masters = True it also keeps a graph-ordered master copy of each
    of the two weight tables (masters()): the in-backward Adam streams it with
    the moments and only WRITES the caller's rows (bbgr_spmm_args.adam_mirror),
    and the next step's forward gathers the master copies through the graph's
    own column indices (bbgr::propagate_rows_graph). A copy is used only while
    its table's version is the one the optimizer left (any other in-place
    write to the weights makes it stale; the next in-backward step rebuilds
    it); it costs one more table of each size in device memory.

    The fused step assumes bpr_loss is the only consumer of the two tables in
    the loss. A gradient that reaches them by another path (e.g. a term
    `lam * W.norm()` added to the loss) lands in .grad and cannot join the
    update already made inside the backward: step() raises on it rather than
    drop it. A parameter is owned by the last FusedAdam(fuse_backward=True)
    built over it; building a second one over a parameter a live one owns
    warns (the first then steps it outside the backward)."""

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, fuse_backward: bool = False):
        if lr < 0.0 or eps < 0.0 or not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError("invalid Adam hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.fuse_backward = bool(fuse_backward)
        self._stepped: set = set()   # ids of parameters stepped in the last backward
        # id(param) -> map[graph row] = caller row: its moments are held in the
        # graph's row order (in-backward steps on an input-order drop-in pair)
        self._graph_rows: dict = {}
        # id(param) -> [graph-ordered copy, its row map, the param's version it matches]
        self._masters: dict = {}
        if self.fuse_backward:
            import weakref
            me = weakref.ref(self)
            for g in self.param_groups:
                for p in g["params"]:
                    e = _IN_BACKWARD.get(id(p))
                    if e is not None and e[0]() is p and e[1]() is not None:
                        warnings.warn("FusedAdam(fuse_backward=True): a parameter owned by "
                                      "another live in-backward FusedAdam moves to this one; "
                                      "the other steps it outside the backward from now on",
                                      RuntimeWarning, stacklevel=2)
                    _IN_BACKWARD[id(p)] = (weakref.ref(p), me)

    def _group_of(self, params):
        for g in self.param_groups:
            ids = {id(p) for p in g["params"]}
            if all(id(p) in ids for p in params):
                return g
        return None

    def _init_state(self, p):
        st = self.state[p]
        if not st:
            st["step"] = torch.tensor(0.0)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return st

    def _to_caller_rows(self, p) -> None:
        """Moments of p back in the caller's row order (if held in the graph's)."""
        m = self._graph_rows.pop(id(p), None)
        if m is None:
            return
        st = self.state[p]
        for k in ("exp_avg", "exp_avg_sq"):
            out = torch.empty_like(st[k])
            out.index_copy_(0, m, st[k])   # caller row m[r] <- graph row r
            st[k] = out

    def _to_graph_rows(self, p, m) -> None:
        """Moments of p in the graph's row order of map m (m[graph row] = caller row)."""
        have = self._graph_rows.get(id(p))
        if have is m:
            return
        self._to_caller_rows(p)
        st = self.state[p]
        for k in ("exp_avg", "exp_avg_sq"):
            st[k] = st[k].index_select(0, m)
        self._graph_rows[id(p)] = m

    def moments(self, p):
        """(exp_avg, exp_avg_sq) of p in the caller's row order (copies when
        they are held in the graph's)."""
        st = self.state[p]
        m = self._graph_rows.get(id(p))
        if m is None:
            return st["exp_avg"], st["exp_avg_sq"]
        out = []
        for k in ("exp_avg", "exp_avg_sq"):
            t = torch.empty_like(st[k])
            t.index_copy_(0, m, st[k])
            out.append(t)
        return tuple(out)

    def state_dict(self):
        """torch's state_dict, moments in the caller's row order."""
        sd = super().state_dict()
        if self._graph_rows:
            index = {}
            for g, gs in zip(self.param_groups, sd["param_groups"]):
                index.update(zip((id(p) for p in g["params"]), gs["params"]))
            for g in self.param_groups:
                for p in g["params"]:
                    if id(p) in self._graph_rows:
                        entry = dict(sd["state"][index[id(p)]])
                        entry["exp_avg"], entry["exp_avg_sq"] = self.moments(p)
                        sd["state"][index[id(p)]] = entry
        return sd

    def load_state_dict(self, state_dict):
        self._graph_rows.clear()   # a loaded state is in the caller's order
        super().load_state_dict(state_dict)

    # True: keep the graph-ordered master copies (off by default: measured at
    # C4, the next forward's first item product gains 1.963 -> 1.888 ms but the
    # user Adam product loses 2.563 -> 2.607 ms — the caller's rows are still
    # written, so the copy adds a 1.28 GB stream where the random read it
    # replaces cost little more; profiles/round6/r6g_masters_ab.txt)
    use_masters = False

    def masters(self, params, row_maps, create: bool = False):
        """The graph-ordered master copies of `params` (copy[r] = p[map[r]]),
        or None unless every one is current with its parameter (same row map,
        the version the optimizer left). create=True builds the missing or
        stale ones from the parameters first."""
        if not self.use_masters:
            return None
        out = []
        for p, m in zip(params, row_maps):
            e = self._masters.get(id(p))
            ok = (e is not None and e[1] is m and e[2] == p._version
                  and e[0].device == p.device and e[0].shape == p.shape)
            if not ok:
                if not create:
                    return None
                e = self._masters[id(p)] = [p.detach().index_select(0, m), m, p._version]
            out.append(e[0])
        return out

    @torch.no_grad()
    def step_in_backward(self, params, run, row_maps=None) -> None:
        """One Adam step of `params` (one param group) carried out by `run(states,
        group, corrections)` inside a backward pass: the step counts advance,
        corrections = [(1 - beta1^t, sqrt(1 - beta2^t)) per parameter] (host
        double, as adam_step), and step() then skips these parameters.
        row_maps (one int64 map per parameter, map[graph row] = caller row):
        `run` takes the moments in the graph's row order."""
        g = self._group_of(params)
        if g is None:
            raise RuntimeError("FusedAdam.step_in_backward: parameters not in one group")
        b1, b2 = g["betas"]
        states, corr = [], []
        for i, p in enumerate(params):
            st = self._init_state(p)
            if row_maps is not None:
                self._to_graph_rows(p, row_maps[i])
            else:
                self._to_caller_rows(p)
            st["step"] += 1
            t = int(st["step"].item())
            states.append(st)
            corr.append((1.0 - b1 ** t, math.sqrt(1.0 - b2 ** t)))
        run(states, g, corr)
        for p in params:
            self._stepped.add(id(p))
            torch.autograd.graph.increment_version(p)
            e = self._masters.get(id(p))
            if e is not None and getattr(run, "masters_updated", False):
                e[2] = p._version   # the copy was updated with the weights
            elif e is not None:
                del self._masters[id(p)]

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if id(p) in self._stepped:   # stepped inside the backward already
                    self._stepped.discard(id(p))
                    # a gradient from another term of the loss cannot join the
                    # update already made: refuse to drop it silently (a zero
                    # .grad from zero_grad(set_to_none=False) is fine)
                    if p.grad is not None and bool(p.grad.ne(0).any()):
                        raise RuntimeError(
                            "FusedAdam(fuse_backward=True): a parameter stepped inside "
                            "the backward also has a .grad from another term of the loss; "
                            "the in-backward step assumes bpr_loss is its only consumer "
                            "(use fuse_backward=False for such losses)")
                    continue
                if p.grad is None:
                    continue
                _lib.require_gpu(p)
                st = self._init_state(p)
                self._to_caller_rows(p)
                st["step"] += 1
                adam_step(p.data, p.grad.contiguous(), st["exp_avg"], st["exp_avg_sq"],
                          int(st["step"].item()), group["lr"], b1, b2, group["eps"],
                          group["weight_decay"])
                # the kernel wrote p through a raw pointer: bump its version as an
                # in-place torch op would, so autograd's saved-tensor checks and
                # the deferred final tables (bbgr.lazy) see the update
                torch.autograd.graph.increment_version(p)
        return loss
