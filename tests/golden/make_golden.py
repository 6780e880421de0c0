"""Generate tests/golden/golden_small.npz from the float64 oracle.

    python tests/golden/make_golden.py

The reference cannot be imported here, so the expected outputs
are the oracle's (oracle/ref_numpy.py, pinned by the hand-derived known
answers in tests/test_oracle.py). The fixture freezes them so that (a) any
change of the oracle shows up in CPU tests and (b) the GPU parity tests on
the box check the HIP path against fixed numbers, not a live recomputation.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import bbgr  # noqa: E402,F401
from bbgr.synthetic import synthetic_credibility, synthetic_edges  # noqa: E402
from oracle import ref_numpy as R  # noqa: E402

U, I, E, DUP, D, K, B = 300, 200, 3000, 30, 64, 3, 256


def build():
    # the last 8 users and 8 items get no edges (isolated rows on both sides)
    e = synthetic_edges(U - 8, I - 8, E, seed=11, items="zipf", duplicates=DUP)
    cred = synthetic_credibility(U, seed=11)
    rng = np.random.default_rng(11)
    u0 = rng.uniform(-1, 1, (U, D)).astype(np.float32)
    i0 = rng.uniform(-1, 1, (I, D)).astype(np.float32)
    gU = rng.normal(size=(U, D)).astype(np.float32)
    gI = rng.normal(size=(I, D)).astype(np.float32)
    users = rng.integers(0, U, B)
    pos = rng.integers(0, I, B)
    neg = rng.integers(0, I, B)
    pop = rng.uniform(0, 1, I).astype(np.float32)
    out = dict(edges=e, cred=cred, u0=u0, i0=i0, gU=gU, gI=gI, users=users, pos=pos,
               neg=neg, pop=pop, meta=np.array([U, I, E, DUP, D, K, B]))
    M_ui, M_iu = R.gs_mats(e, U, I, cred)
    uf, itf, _, _ = R.propagate_gs(M_ui, M_iu, u0, i0, K)
    gu0, gi0 = R.backward_gs(M_ui, M_iu, gU, gI, K)
    out.update(gs_uf=uf, gs_if=itf, gs_gu0=gu0, gs_gi0=gi0)
    A_ui, A_iu = R.gs_mats(e, U, I, cred, method_a=True)
    uf, itf, _, _ = R.propagate_gs(A_ui, A_iu, u0, i0, K)
    out.update(ma_uf=uf, ma_if=itf)
    Mj_iu, Mj_ui, _ = R.j_mats(e, U, I, cred)
    uf, itf, _, _ = R.propagate_j(Mj_iu, Mj_ui, u0, i0, K)
    gu0, gi0 = R.backward_j(Mj_iu, Mj_ui, gU, gI, K)
    out.update(j_uf=uf, j_if=itf, j_gu0=gu0, j_gi0=gi0)
    S = R.sym_values(e, U, I)
    x0 = np.concatenate([u0, i0])
    xf, _ = R.propagate_sym(S, x0, K)
    gx = R.backward_sym(S, np.concatenate([gU, gI]), K)
    out.update(sym_xf=xf, sym_gx=gx)
    uf, itf = out["gs_uf"], out["gs_if"]
    loss, g = R.bpr_loss(uf, itf, u0, i0, users, pos, neg, 1e-4, pop, 0.05)
    out.update(bpr_loss=np.array(loss), bpr_g_uf=g["g_uf"], bpr_g_if=g["g_if"],
               bpr_g_ue=g["g_ue"], bpr_g_ie=g["g_ie"])
    p, m, v = R.adam_step(u0, gU, np.zeros_like(u0), np.zeros_like(u0), 1)
    out.update(adam_p1=p)
    for k, val in list(out.items()):
        if isinstance(val, np.ndarray) and val.dtype == np.float64 and val.ndim == 2:
            out[k] = val.astype(np.float32)
    return out


if __name__ == "__main__":
    np.savez_compressed(os.path.join(HERE, "golden_small.npz"), **build())
    print("wrote", os.path.join(HERE, "golden_small.npz"))
