"""GPU cosine top-k (csrc/search.hip, latice.index.faiss_db) vs the float64 restatement of
the reference's IndexFlatIP search (oracle/index_oracle.py).  Scores within 2e-6 (fp32
products of unit vectors); ids must match wherever the k-th and (k+1)-th oracle scores are
further apart than that tolerance."""
import numpy as np
import pytest
import torch

from latice.index import faiss_db as F
from oracle import index_oracle as IO

pytestmark = pytest.mark.gpu
STOL = 2e-6


def _check(db, q, k):
    dbn = F.l2_normalize(torch.from_numpy(db).cuda())
    qn = F.l2_normalize(torch.from_numpy(q).cuda())
    s, i = F.cosine_topk(dbn, qn, k)
    s, i = s.cpu().numpy(), i.cpu().numpy()
    rs, ri = IO.cosine_topk(IO.l2_normalize(db), IO.l2_normalize(q), min(k + 1, db.shape[0]))
    assert np.abs(s - rs[:, :k]).max() <= STOL
    assert np.all(np.diff(s, axis=1) <= 0)                      # best first
    for r in range(q.shape[0]):
        gap = rs[r, k - 1] - rs[r, k] if rs.shape[1] > k else 1.0
        if gap > 2 * STOL:
            assert set(i[r]) == set(ri[r, :k]), r
    return s, i


def test_l2_normalize_matches_reference_formula(cuda):
    rng = np.random.default_rng(1)
    v = rng.standard_normal((1000, 16)).astype(np.float32)
    v[7] = 0.0   # zero rows stay zero (norm 0 -> 1)
    out = F.l2_normalize(torch.from_numpy(v).cuda()).cpu().numpy()
    assert np.abs(out - IO.l2_normalize(v)).max() < 1e-6
    assert np.all(out[7] == 0)


@pytest.mark.parametrize("n,d,Q,k", [(20000, 16, 37, 20), (4096, 16, 1, 1), (777, 32, 9, 64),
                                     (64, 16, 5, 64), (130, 64, 3, 17), (100003, 16, 70, 20)])
def test_cosine_topk_matches_oracle(cuda, n, d, Q, k):
    rng = np.random.default_rng(n + d + Q + k)
    db = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal((Q, d)).astype(np.float32)
    _check(db, q, k)


def test_cosine_topk_ties_break_to_lower_row(cuda):
    rng = np.random.default_rng(5)
    db = rng.standard_normal((3000, 16)).astype(np.float32)
    q = rng.standard_normal((4, 16)).astype(np.float32)
    db[2999] = db[2500] = db[11] = q[0]   # three bit-identical best rows for query 0
    s, i = _check(db, q, 5)
    assert list(i[0, :3]) == [11, 2500, 2999]


def test_database_api(cuda, tmp_path):
    rng = np.random.default_rng(9)
    cfg = F.FaissLatentVectorDatabaseConfig(npz_path=str(tmp_path / "idx.npz"), dimension=16)
    db = F.FaissLatentVectorDatabase(cfg)
    assert db.get_count() == 0
    d, i = db.query_similar(rng.standard_normal(16).astype(np.float32))
    assert d.size == 0 and i.size == 0
    lv = rng.standard_normal((500, 16)).astype(np.float64)
    ori = rng.uniform(0, 360, (500, 3))
    db.add_vectors(lv[:300], ori[:300])
    db.add_vectors(torch.from_numpy(lv[300:]).cuda(), ori[300:])   # device tensors stay on device
    assert db.get_count() == 500
    with pytest.raises(ValueError):
        db.add_vectors(lv[:3, :8], ori[:3])
    q = lv[42] + 1e-3 * rng.standard_normal(16)
    d, i = db.query_similar(q, n_results=20)
    assert i[0] == 42 and d.shape == (20,) and i.dtype == np.int64
    with pytest.raises(ValueError):
        db.query_similar_batch(lv[:10], n_results=100)               # > the GPU top-k limit
    d, i = db.query_similar_batch(lv[:10], n_results=5)
    assert d.shape == (10, 5) and np.array_equal(i[:, 0], np.arange(10))
    small = F.FaissLatentVectorDatabase(F.FaissLatentVectorDatabaseConfig(
        npz_path=str(tmp_path / "small.npz"), dimension=16))
    small.add_vectors(lv[:7], ori[:7])
    d, i = small.query_similar(lv[3], n_results=20)                  # fewer rows than asked
    assert d.shape == (7,) and sorted(i) == list(range(7)) and i[0] == 3
    db.save()
    db2 = F.FaissLatentVectorDatabase(cfg)
    assert db2.get_count() == 500
    d2, i2 = db2.query_similar(q, n_results=20)
    assert np.array_equal(i2, db.query_similar(q, n_results=20)[1])
    db2.delete_persistence()
    assert db2.get_count() == 0


def _cluster_db(rng, n_clusters=40, per=24, noise_deg=0.3, dim=16):
    """Latents clustered per orientation; orientations noisy around cluster centres, some
    copies hidden behind random cubic symmetry operators."""
    from scipy.spatial.transform import Rotation as R
    sym = R.from_quat(IO.CUBIC_SYMMETRY)
    lat, ori = [], []
    for c in range(n_clusters):
        centre = R.random(random_state=int(rng.integers(1 << 30)))
        z = rng.standard_normal(dim)
        for j in range(per):
            rot = R.from_rotvec(np.radians(noise_deg) * rng.standard_normal(3)) * centre
            if j % 7 == 3:
                rot = sym[int(rng.integers(24))] * rot
            ori.append(rot.as_euler("zxz", degrees=True))
            lat.append(z + 0.05 * rng.standard_normal(dim))
    return np.array(lat, np.float32), np.array(ori)


@pytest.mark.parametrize("thr,minm,maxit", [(1.0, 18, 3), (2.0, 12, 3), (1.0, 15, 2), (5.0, 1, 1), (0.5, 21, 3)])
def test_orientation_consensus_matches_oracle(cuda, thr, minm, maxit):
    rng = np.random.default_rng(int(thr * 10) + minm + maxit)
    lat, ori = _cluster_db(rng)
    db = F.FaissLatentVectorDatabase(F.FaissLatentVectorDatabaseConfig(npz_path="/nonexistent/x.npz"))
    db.add_vectors(lat, ori)
    queries = lat[::9] + 0.02 * rng.standard_normal((len(lat[::9]), 16)).astype(np.float32)
    res = db.find_best_orientations_batch(queries, top_n=20, orientation_threshold=thr,
                                          min_required_matches=minm, max_iterations=maxit)
    n_ok = 0
    for r in res:
        best, mean, ok, sim = IO.find_best_orientation(r.candidate_orientations, thr, minm, maxit)
        assert r.success == ok
        assert np.array_equal(r.similar_indices, sim)
        if ok:
            n_ok += 1
            # same rotation; Euler angles compared modulo 360 (wrap at +-180)
            d = (np.asarray(r.best_orientation) - best + 180.0) % 360.0 - 180.0
            assert np.abs(d).max() < 1e-6, (r.best_orientation, best)
            assert r.mean_orientation is not None
        else:
            assert r.mean_orientation is None and np.array_equal(r.best_orientation, best)
    assert n_ok > 0 or minm > 20   # more required matches than candidates: never


def test_single_query_api_and_empty_index(cuda):
    rng = np.random.default_rng(11)
    lat, ori = _cluster_db(rng, n_clusters=5)
    db = F.FaissLatentVectorDatabase(F.FaissLatentVectorDatabaseConfig(npz_path="/nonexistent/y.npz"))
    r = db.find_best_orientation(lat[0])
    assert not r.success and np.isnan(r.best_orientation).all()
    db.add_vectors(lat, ori)
    r = db.find_best_orientation(lat[0], top_n=20, orientation_threshold=2.0, min_required_matches=10)
    best, mean, ok, sim = IO.find_best_orientation(r.candidate_orientations, 2.0, 10, 3)
    assert r.success == ok and r.candidate_orientations.shape == (20, 3) and r.distances.shape == (20,)
