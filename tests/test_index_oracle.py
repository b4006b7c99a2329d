"""CPU checks of oracle/index_oracle.py: the search restatement's ordering and the zxz
Euler convention the consensus kernel (csrc/orient.hip) restates, pinned to scipy (the
reference's dependency for latice/index/faiss_db.py:258-398)."""
import warnings

import numpy as np
from scipy.spatial.transform import Rotation as R

from oracle import index_oracle as IO


def test_topk_orders_by_score_then_row():
    db = np.array([[1, 0], [0, 1], [1, 0], [0.6, 0.8]], float)
    s, i = IO.cosine_topk(IO.l2_normalize(db), np.array([[1.0, 0.0]]), 3)
    assert list(i[0]) == [0, 2, 3] and np.allclose(s[0], [1, 1, 0.6])


def _qmul(p, q):
    v = p[..., 3:] * q[..., :3] + q[..., 3:] * p[..., :3] + np.cross(p[..., :3], q[..., :3])
    w = p[..., 3:] * q[..., 3:] - np.sum(p[..., :3] * q[..., :3], -1, keepdims=True)
    return np.concatenate([v, w], -1)


def _from_euler_zxz(e):   # the kernel's formula, csrc/orient.hip from_euler_zxz
    a, b, c = np.radians(e).T
    z = np.zeros_like(a)
    qa = np.stack([z, z, np.sin(a / 2), np.cos(a / 2)], -1)
    qb = np.stack([np.sin(b / 2), z, z, np.cos(b / 2)], -1)
    qc = np.stack([z, z, np.sin(c / 2), np.cos(c / 2)], -1)
    return _qmul(qc, _qmul(qb, qa))


def _as_euler_zxz(q):     # the kernel's formula, csrc/orient.hip as_euler_zxz
    a, b, c, d = q[:, 3], q[:, 2], q[:, 0], q[:, 1]
    ang = np.zeros((len(q), 3))
    ang[:, 1] = 2 * np.arctan2(np.hypot(c, d), np.hypot(a, b))
    hs, hd = np.arctan2(b, a), np.arctan2(d, c)
    c1, c2 = np.abs(ang[:, 1]) <= 1e-7, np.abs(ang[:, 1] - np.pi) <= 1e-7
    c0 = ~(c1 | c2)
    ang[:, 0] = np.where(c0, hs - hd, np.where(c1, 2 * hs, -2 * hd))
    ang[:, 2] = np.where(c0, hs + hd, 0)
    ang = np.where(ang < -np.pi, ang + 2 * np.pi, np.where(ang > np.pi, ang - 2 * np.pi, ang))
    return np.degrees(ang)


def test_kernel_euler_formulas_match_scipy():
    rng = np.random.default_rng(0)
    e = np.stack([rng.uniform(-180, 180, 3000), rng.uniform(0, 180, 3000),
                  rng.uniform(-180, 180, 3000)], 1)
    assert np.abs(_from_euler_zxz(e) - R.from_euler("zxz", e, degrees=True).as_quat()).max() < 1e-15
    r = R.from_quat(rng.standard_normal((3000, 4)))
    assert np.abs(_as_euler_zxz(r.as_quat()) - r.as_euler("zxz", degrees=True)).max() < 1e-9
    g = np.array([[30, 0, 0], [10, 0, 20], [50, 180, -30], [10, 1e-9, 5], [-170, 180, 170]], float)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")   # scipy warns on gimbal lock
        rg = R.from_euler("zxz", g, degrees=True)
        assert np.abs(_as_euler_zxz(rg.as_quat()) - rg.as_euler("zxz", degrees=True)).max() < 1e-9


def test_consensus_oracle_averages_the_cluster():
    """20 noisy copies of one orientation: the raw misorientation test (no symmetry, as the
    reference does at faiss_db.py:313-318) groups them, the mean lands near the truth."""
    rng = np.random.default_rng(3)
    base = R.from_euler("zxz", [40, 30, 60], degrees=True)
    cand = [(R.from_rotvec(np.radians(0.2) * rng.standard_normal(3)) * base).as_euler("zxz", degrees=True)
            for _ in range(20)]
    best, mean, ok, sim = IO.find_best_orientation(np.array(cand), orientation_threshold=2.0,
                                                   min_required_matches=18)
    assert ok and len(sim) == 20
    d = (R.from_euler("zxz", best, degrees=True).inv() * base).magnitude()
    assert np.degrees(d) < 0.2
