"""ORACLE — test infrastructure, NOT product code.

Float64 K-layer LightGCN chains at the BASELINE sizes, on the host
(oracle/csrc/chain64.c through ctypes): the reference's propagation
(Version-2/lighgcn_cu_pop.py:472-490 Gauss-Seidel, lightgcn_cu.py:420-448
Jacobi) and its autograd adjoint, from given fp32 u0 / i0, in float64, with
the reference's fp32 operator values (oracle/ref_numpy.edge_weights). Used by
tests/test_gpu_fullsize.py so every full-size check compares the GPU with a
chain evaluated from the SAME inputs, never with the GPU's own intermediates.

Memory: the tables are float64 numpy arrays (C4: 2.6 GB per user table; C5:
20 GB), the two CSRs 12 B per edge each.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import native
from . import ref_numpy as R


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _lib():
    L = native.lib()
    if not getattr(L, "_chain64_bound", False):
        P, I64, I32, D = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_double
        L.oracle_csr_perm.argtypes = [I64, P, I64, P, P]
        L.oracle_csr_perm.restype = ctypes.c_int
        L.oracle_spmm64.argtypes = [I64, P, P, P, P, I64, I32, P, I64, P, I64, D, P, I64]
        L.oracle_spmm64.restype = None
        L._chain64_bound = True
    return L


class Csr64:
    """One side's CSR of the edge list (rows = that endpoint), with the fp32
    values of one or more operators in CSR slot order."""

    def __init__(self, rows: np.ndarray, cols: np.ndarray, n_rows: int, **weights):
        rows = np.ascontiguousarray(rows, np.int32)
        E = rows.size
        self.n_rows = int(n_rows)
        self.indptr = np.empty(self.n_rows + 1, np.int64)
        perm = np.empty(max(E, 1), np.int64)
        rc = _lib().oracle_csr_perm(E, _p(rows), self.n_rows, _p(self.indptr), _p(perm))
        if rc != 0:
            raise ValueError(f"oracle_csr_perm failed ({rc})")
        perm = perm[:E]
        self.cols = np.ascontiguousarray(np.asarray(cols)[perm], np.int32)
        self.w = {k: np.ascontiguousarray(np.asarray(v)[perm], np.float32)
                  for k, v in weights.items()}

    def degrees(self) -> np.ndarray:
        return np.diff(self.indptr)

    def mm(self, which: str, x: np.ndarray, out=None, add=None, add_scale: float = 1.0,
           acc=None) -> np.ndarray:
        """out = add_scale*add + M x (float64), acc += out; returns out (None if
        out is False: only acc is updated)."""
        d = x.shape[1]
        assert x.dtype == np.float64 and x.flags.c_contiguous
        if out is None:
            out = np.empty((self.n_rows, d), np.float64)
        y = None if out is False else out
        for t in (y, add, acc):
            assert t is None or (t.dtype == np.float64 and t.flags.c_contiguous
                                 and t.shape == (self.n_rows, d))
        _lib().oracle_spmm64(self.n_rows, _p(self.indptr), _p(self.cols), _p(self.w[which]),
                             _p(x), d, d, None if y is None else _p(y), d,
                             None if add is None else _p(add), d, float(add_scale),
                             None if acc is None else _p(acc), d)
        return y


class Chain64:
    """The bipartite operator pair of one reference family on an edge list.

    kind "gs" / "method_a" (Version-2 / version_1 long-tail): M_ui [U x I]
    (user<-item, values w_base) and M_iu [I x U] (item<-user, c_u * w_base);
    kind "j" (lightgcn_cu.py, names swapped there): item<-user c_u/denom,
    user<-item 1/denom. `user` / `item` are the CSRs whose rows are users /
    items; each holds the forward operator's values ("fwd") and the values of
    the other direction's operator, whose transpose it is ("bwd")."""

    def __init__(self, edges_2xE: np.ndarray, U: int, I: int, kind: str, cred=None):
        self.U, self.I, self.kind = int(U), int(I), kind
        deg_u, deg_i = R.degrees(edges_2xE, U, I)
        w_user_from_item, w_item_from_user = R.edge_weights(kind, edges_2xE[0], edges_2xE[1],
                                                            deg_u, deg_i, cred)
        self.user = Csr64(edges_2xE[0], edges_2xE[1], U, fwd=w_user_from_item,
                          bwd=w_item_from_user)
        self.item = Csr64(edges_2xE[1], edges_2xE[0], I, fwd=w_item_from_user,
                          bwd=w_user_from_item)
        del w_user_from_item, w_item_from_user
        self.deg_u, self.deg_i = deg_u, deg_i

    # -- forward ----------------------------------------------------------------
    def forward(self, u0: np.ndarray, i0: np.ndarray, K: int, order: str, keep_u=None,
                keep_i=None):
        """Final tables (layer means, float64) and the rows keep_u / keep_i of
        every layer k = 0..K: (u_final, i_final, [u_k[keep_u]], [i_k[keep_i]]).
        order "gs": i_k = M_iu u_{k-1}; u_k = M_ui i_k (Version-2:482-487).
        order "jacobi": i_k = M_iu u_{k-1}; u_k = M_ui i_{k-1} (cu:429-447)."""
        u = np.ascontiguousarray(u0, np.float64)
        i = np.ascontiguousarray(i0, np.float64)
        acc_u, acc_i = u.copy(), i.copy()
        lay_u = [u[keep_u]] if keep_u is not None else []
        lay_i = [i[keep_i]] if keep_i is not None else []
        for _ in range(int(K)):
            i_new = self.item.mm("fwd", u, acc=acc_i)
            u_new = self.user.mm("fwd", i_new if order == "gs" else i, acc=acc_u)
            u, i = u_new, i_new
            if keep_u is not None:
                lay_u.append(u[keep_u])
            if keep_i is not None:
                lay_i.append(i[keep_i])
        del u, i
        acc_u /= (K + 1)
        acc_i /= (K + 1)
        return acc_u, acc_i, lay_u, lay_i

    # -- backward (autograd adjoint of the forward; oracle/ref_numpy.backward_*) --
    def backward(self, gU: np.ndarray, gI: np.ndarray, K: int, order: str):
        """(grad u0, grad i0) in float64 given dL/d(u_final), dL/d(i_final)."""
        gl = 1.0 / (K + 1)
        gU = np.ascontiguousarray(gU, np.float64) * gl
        gI = np.ascontiguousarray(gI, np.float64) * gl
        if order == "gs":     # Gi = gI' + M_ui^T Gu ; Gu = gU' + M_iu^T Gi
            Gu = gU.copy()
            for _ in range(int(K)):
                Gi = self.item.mm("bwd", Gu, add=gI)
                Gu = self.user.mm("bwd", Gi, add=gU)
            return Gu, gI
        Gu, Gi = gU.copy(), gI.copy()   # jacobi: Gu' = gU'+M_ui^T... (ref_numpy.backward_j)
        for _ in range(int(K)):
            Gu, Gi = self.user.mm("bwd", Gi, add=gU), self.item.mm("bwd", Gu, add=gI)
        return Gu, Gi
