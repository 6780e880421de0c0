"""Generate tests/golden/sampler_c4_b8192.npz: the first training batch of a
seeded Version-2 run on the C4 graph, drawn by the reference's own per-user
sampler loop as the oracle restates it (oracle/ref_numpy.py
sample_batch_reference_style = Version-2/lighgcn_cu_pop.py:835-849 with
sample_pos_item :339-343, sample_neg_item_popmix :349-376, user_has_item
:330-336, numpy's Generator.choice(p=) for every popularity draw).

    python tests/golden/make_golden_sampler.py      (~1 min: 1M-item choice per draw)

The run's own order (V2:795-821): rng = np.random.default_rng(42);
train_users = users with >= 1 train edge; rng.shuffle(train_users); the first
batch is train_users[:8192] (BASELINE C4's batch); pop_prob from the train
item degrees with gamma 0.75 (:805-810), mix_pop 0.7, max_tries 50 (CFG).
Stored: the batch users, the (used, pos, neg) arrays and the Generator's
bit_generator.state after the loop (JSON text), so a test can check that a
sampler consumed exactly the same random bits.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import bbgr  # noqa: E402,F401
from bbgr.synthetic import CONFIGS, config_edges  # noqa: E402
from oracle import ref_numpy as R  # noqa: E402

BATCH = 8192


def c4_first_batch_inputs(with_edges: bool = False):
    """(indptr, indices, batch_users, num_items, pop_prob, rng after the
    shuffle[, edges]) of a seeded V2 run on the C4 graph (shared with the test)."""
    c = CONFIGS["C4"]
    U, I = c["num_users"], c["num_items"]
    e = config_edges("C4")
    indptr, indices = R.edges_to_user_csr(e, U)
    pp = R.pop_prob(e, I)
    rng = np.random.default_rng(42)
    train_users = np.where((indptr[1:] - indptr[:-1]) > 0)[0]
    rng.shuffle(train_users)
    out = (indptr, indices, train_users[:BATCH].copy(), I, pp, rng)
    return out + (e,) if with_edges else out


def main():
    indptr, indices, users, I, pp, rng = c4_first_batch_inputs()
    used, pos, neg = R.sample_batch_reference_style(indptr, indices, users, I, rng, pp,
                                                    mix_pop=0.7, max_tries=50)
    out = os.path.join(HERE, "sampler_c4_b8192.npz")
    np.savez_compressed(out, batch_users=users.astype(np.int64), used=used.astype(np.int64),
                        pos=pos.astype(np.int64), neg=neg.astype(np.int64),
                        state=np.array(json.dumps(rng.bit_generator.state)))
    print("wrote", out, used.size)


if __name__ == "__main__":
    main()
