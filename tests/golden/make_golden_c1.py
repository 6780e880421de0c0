"""Generate tests/golden/golden_c1.npz: the BASELINE C1 workload (ML-100K
scale: 943 users x 1682 items, 100,000 edges, d=64, K=3) through the float64
oracle, as SURVEY §8(c)(ii) asks.

    python tests/golden/make_golden_c1.py

C1 is the reference's own CPU case, lightgcn.py (symmetric normalised
adjacency, lightgcn.py:318-372), so that path is frozen layer by layer: every
propagated layer x_1..x_K, the layer mean, the BPR loss of one batch
(lightgcn.py:333-349: ego rows of emb.weight, items offset by U) and the
gradient of emb.weight through the whole chain. The other operator families
(GS / Method A / Jacobi, Beta credibility) are frozen as final tables of the
same inputs. Stored as float32 (the float64 oracle rounded once: 6e-8
relative, far inside the 1e-5 parity bar).

The reference cannot be imported here: the expected values are
the oracle's, pinned by the hand-derived known answers in tests/test_oracle.py.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import bbgr  # noqa: E402,F401
from bbgr.synthetic import (CONFIGS, CONFIG_SEED, config_edges,  # noqa: E402
                            synthetic_credibility, xavier_tables)
from oracle import ref_numpy as R  # noqa: E402

REG = 1e-4


def build():
    c = CONFIGS["C1"]
    U, I, D, K = c["num_users"], c["num_items"], c["emb_dim"], c["num_layers"]
    e = config_edges("C1")
    cred = synthetic_credibility(U, CONFIG_SEED["C1"], "beta")
    u0, i0 = xavier_tables(U, I, D, seed=42)
    rng = np.random.default_rng(CONFIG_SEED["C1"])
    # one reference batch: B = 4096 > 943 users, so the slice of the epoch
    # permutation is every train user once (lightgcn.py:574-585); one
    # positive from the user's row, one uniform item as the negative
    users = rng.permutation(np.unique(e[0])).astype(np.int64)
    indptr, indices = R.edges_to_user_csr(e, U)
    pos = np.array([R.sample_pos_item(indptr, indices, int(u), rng) for u in users], np.int64)
    neg = np.array([R.sample_neg_item(indptr, indices, int(u), I, rng) for u in users], np.int64)
    out = dict(edges=e, cred=cred, u0=u0, i0=i0, users=users, pos=pos, neg=neg,
               meta=np.array([U, I, e.shape[1], D, K]))
    # lightgcn.py: symmetric A_hat on [N, d], every layer
    S = R.sym_values(e, U, I)
    x0 = np.concatenate([u0, i0])
    xf, xs = R.propagate_sym(S, x0, K)
    for k in range(1, K + 1):
        out[f"sym_x{k}"] = xs[k]
    out["sym_xf"] = xf
    loss, g = R.bpr_loss(xf[:U], xf[U:], u0, i0, users, pos, neg, REG)
    gx = R.backward_sym(S, np.concatenate([g["g_uf"], g["g_if"]]), K)
    gx = gx + np.concatenate([g["g_ue"], g["g_ie"]])      # ego L2 rows of emb.weight
    out.update(sym_loss=np.array(loss), sym_grad_emb=gx)
    # the other families on the same inputs: final tables
    M_ui, M_iu = R.gs_mats(e, U, I, cred)
    uf, itf, _, _ = R.propagate_gs(M_ui, M_iu, u0, i0, K)
    out.update(gs_uf=uf, gs_if=itf)
    A_ui, A_iu = R.gs_mats(e, U, I, cred, method_a=True)
    uf, itf, _, _ = R.propagate_gs(A_ui, A_iu, u0, i0, K)
    out.update(ma_uf=uf, ma_if=itf)
    Mj_iu, Mj_ui, _ = R.j_mats(e, U, I, cred)
    uf, itf, _, _ = R.propagate_j(Mj_iu, Mj_ui, u0, i0, K)
    out.update(j_uf=uf, j_if=itf)
    for k, val in list(out.items()):
        if isinstance(val, np.ndarray) and val.dtype == np.float64 and val.ndim == 2:
            out[k] = val.astype(np.float32)
    return out


if __name__ == "__main__":
    np.savez_compressed(os.path.join(HERE, "golden_c1.npz"), **build())
    print("wrote", os.path.join(HERE, "golden_c1.npz"))
