"""CPU: ingest of the reference's on-disk formats (synthetic files written here)."""
import numpy as np
import pytest

from bbgr import ingest
from bbgr.synthetic import synthetic_edges


def test_train_edges_npy_roundtrip_memmapped(tmp_path):
    e = synthetic_edges(50, 30, 400, 1)
    np.save(tmp_path / "train_edges.npy", e)
    got = ingest.load_edges_npy(tmp_path / "train_edges.npy")
    assert isinstance(got, np.memmap)
    np.testing.assert_array_equal(got, e)
    np.save(tmp_path / "bad.npy", e.astype(np.int64))
    with pytest.raises(ValueError, match="int32"):
        ingest.load_edges_npy(tmp_path / "bad.npy")
    np.save(tmp_path / "bad2.npy", e[:1])
    with pytest.raises(ValueError, match="shape"):
        ingest.load_edges_npy(tmp_path / "bad2.npy")


def test_u2i_memmaps(tmp_path):
    E = 123
    rng = np.random.default_rng(0)
    src = rng.integers(0, 40, E).astype(np.int32)
    dst = rng.integers(0, 20, E).astype(np.int32)
    attr = rng.random((E, 5)).astype(np.float32)
    for name, arr in (("u2i_src.mmap", src), ("u2i_dst.mmap", dst), ("u2i_attr.mmap", attr)):
        m = np.memmap(tmp_path / name, dtype=arr.dtype, mode="w+", shape=arr.shape)
        m[:] = arr
        m.flush()
    s, d, a = ingest.load_u2i_memmap(tmp_path, with_attr=True)
    np.testing.assert_array_equal(s, src)
    np.testing.assert_array_equal(d, dst)
    np.testing.assert_array_equal(a, attr)


def test_to_device_streams_in_chunks():
    a = np.arange(1000, dtype=np.int32)
    t = ingest.to_device_i32(a, "cpu", chunk=64)
    assert t.tolist() == a.tolist()
    u, i = ingest.edges_to_device(np.stack([a, a[::-1]]), "cpu")
    assert i[0].item() == 999


def test_credibility_csv_semantics(tmp_path):
    p = tmp_path / "cred.csv"
    p.write_text("user_id,credibility\nalice,0.25\nbob,7.0\nzed,0.5\ncarol,oops\n")
    c = ingest.load_credibility_csv(p, 4, {"alice": 0, "bob": 1, "carol": 2})
    np.testing.assert_allclose(c, [0.25, 1.0, 1.0, 1.0])        # clipped; defaults 1.0
    p2 = tmp_path / "cred2.csv"
    p2.write_text("user_idx,credibility\n3,-1\n1,0.75\n9,0.1\n")
    np.testing.assert_allclose(ingest.load_credibility_csv(p2, 4), [1.0, 0.75, 1.0, 0.0])
    p3 = tmp_path / "cred3.csv"
    p3.write_text("uid,score\nx,1\n")
    with pytest.raises(ValueError, match="Unsupported cred CSV header"):
        ingest.load_credibility_csv(p3, 4)
    np.testing.assert_allclose(ingest.load_credibility_csv(tmp_path / "missing.csv", 2), [1, 1])


def test_credibility_npy(tmp_path):
    np.save(tmp_path / "c.npy", np.array([0.5, 2.0, -1.0]))
    np.testing.assert_allclose(ingest.load_credibility_npy(tmp_path / "c.npy", 3), [0.5, 1, 0])
    with pytest.raises(ValueError):
        ingest.load_credibility_npy(tmp_path / "c.npy", 4)


def test_degree_relabel_orders_and_maps_back():
    """ingest.degree_relabel: degrees non-increasing in the new ids, ties by
    ascending original id, the maps invert the renumbering, and the edge
    multiset is the original one under the maps."""
    U, I = 300, 120
    e = synthetic_edges(U, I, 4000, 7, items="zipf")
    e2, uid, iid = ingest.degree_relabel(e, U, I)
    assert e2.dtype == np.int32 and e2.shape == e.shape
    du = np.bincount(e2[0], minlength=U)
    di = np.bincount(e2[1], minlength=I)
    assert (np.diff(du) <= 0).all() and (np.diff(di) <= 0).all()
    np.testing.assert_array_equal(uid[e2[0]], e[0])
    np.testing.assert_array_equal(iid[e2[1]], e[1])
    assert sorted(uid.tolist()) == list(range(U)) and sorted(iid.tolist()) == list(range(I))
    d0 = np.bincount(e[0], minlength=U)
    for a in range(U - 1):   # equal degrees keep ascending original ids
        if d0[uid[a]] == d0[uid[a + 1]]:
            assert uid[a] < uid[a + 1]
    with pytest.raises(ValueError):
        ingest.degree_relabel(e, U - 1, I)
