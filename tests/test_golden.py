"""CPU: the oracle still reproduces the committed golden fixture."""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def test_oracle_reproduces_golden():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    fresh = mg.build()
    gold = np.load(os.path.join(HERE, "golden", "golden_small.npz"))
    assert set(gold.files) == set(fresh)
    for k in gold.files:
        a, b = gold[k], fresh[k]
        if a.dtype.kind in "iu":
            np.testing.assert_array_equal(a, b, err_msg=k)
        else:
            np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7, err_msg=k)


def test_golden_edges_have_duplicates_and_isolated_rows():
    g = np.load(os.path.join(HERE, "golden", "golden_small.npz"))
    U, I, E, DUP = (int(x) for x in g["meta"][:4])
    e = g["edges"]
    assert e.shape == (2, E + DUP)
    keys = e[0].astype(np.int64) * I + e[1]
    assert np.unique(keys).size < keys.size            # duplicate pairs present
    assert (np.bincount(e[1], minlength=I) == 0).sum() >= 8   # isolated items
    assert (np.bincount(e[0], minlength=U) == 0).sum() >= 8   # isolated users


def test_oracle_reproduces_golden_c1():
    """The C1 fixture (BASELINE configs[0], lightgcn.py path) is still what the
    oracle computes."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "make_golden_c1", os.path.join(HERE, "golden", "make_golden_c1.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    fresh = mg.build()
    gold = np.load(os.path.join(HERE, "golden", "golden_c1.npz"))
    assert set(gold.files) == set(fresh)
    for k in gold.files:
        a, b = gold[k], fresh[k]
        if a.dtype.kind in "iu":
            np.testing.assert_array_equal(a, b, err_msg=k)
        else:
            np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7, err_msg=k)
    U, I, E, d, K = (int(x) for x in gold["meta"])
    assert (U, I, E, d, K) == (943, 1682, 100_000, 64, 3)
    # every train user once, positives from the row, negatives outside it
    e = gold["edges"]
    assert np.array_equal(np.sort(gold["users"]), np.unique(e[0]))
    keys = set((e[0].astype(np.int64) * I + e[1]).tolist())
    assert all(int(u) * I + int(p) in keys for u, p in zip(gold["users"], gold["pos"]))
    assert not any(int(u) * I + int(n) in keys for u, n in zip(gold["users"], gold["neg"]))
