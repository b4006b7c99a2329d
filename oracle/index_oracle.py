"""CPU restatement of the reference's latent-dictionary search and orientation consensus
(TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker, never by the product path).

Search (latice/index/faiss_db.py): rows and queries are L2-normalised (`_l2_normalize`,
faiss_db.py:107-111: norm 0 -> 1) and searched exhaustively by inner product
(faiss.IndexFlatIP via index_factory "Flat" + METRIC_INNER_PRODUCT, faiss_db.py:134-138;
`query_similar` :216-256 returns the k best scores and row ids).  faiss-cpu 1.10 is not
installed here, so parity with faiss itself is unpinned; the search is exact, so this float64
restatement differs from any fp32 implementation only by summation rounding.  Ties are
ordered by the lower row id (faiss leaves the order of equal scores unspecified).
"""
from __future__ import annotations

import numpy as np


def l2_normalize(v: np.ndarray) -> np.ndarray:
    """faiss_db.py:107-111 in float64."""
    v = np.asarray(v, dtype=np.float64)
    n = np.linalg.norm(v, axis=1, keepdims=True)
    n[n == 0] = 1.0
    return v / n


def cosine_topk(db_normed: np.ndarray, q_normed: np.ndarray, k: int):
    """Exhaustive inner-product top-k (scores desc, row id asc): (scores (Q,k), ids (Q,k))."""
    s = np.asarray(q_normed, np.float64) @ np.asarray(db_normed, np.float64).T
    ids = np.argsort(-s, axis=1, kind="stable")[:, :k]
    return np.take_along_axis(s, ids, 1), ids


# ----------------------------------------------------------------------------- consensus
# latice/utils/constants.py:13-39 (scalar-last quaternions, as scipy's Rotation.from_quat)
_S2 = 1 / np.sqrt(2)
CUBIC_SYMMETRY = np.array([
    [1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1],
    [0.5, 0.5, 0.5, 0.5], [0.5, -0.5, -0.5, -0.5], [0.5, 0.5, -0.5, 0.5], [0.5, -0.5, 0.5, -0.5],
    [0.5, -0.5, 0.5, 0.5], [0.5, 0.5, -0.5, -0.5], [0.5, -0.5, -0.5, 0.5], [0.5, 0.5, 0.5, -0.5],
    [_S2, _S2, 0, 0], [_S2, 0, _S2, 0], [_S2, 0, 0, _S2], [_S2, -_S2, 0, 0], [_S2, 0, -_S2, 0],
    [_S2, 0, 0, -_S2], [0, _S2, _S2, 0], [0, -_S2, _S2, 0], [0, 0, _S2, _S2], [0, 0, -_S2, _S2],
    [0, _S2, 0, _S2], [0, -_S2, 0, _S2]])


def find_best_orientation(candidates_euler, orientation_threshold=1.0, min_required_matches=18,
                          max_iterations=3):
    """latice/index/faiss_db.py:258-372 (== chroma_db.py:261-375) on one query's candidate
    orientations (top-n order, ZXZ Euler degrees), with scipy Rotation as the reference uses
    it.  Returns (best (3,), mean (3,) or None, success, similar_indices)."""
    from scipy.spatial.transform import Rotation as R
    quat_sym = R.from_quat(CUBIC_SYMMETRY)
    cand = np.asarray(candidates_euler, np.float64)
    rotations = R.from_euler("zxz", cand, degrees=True)
    success, best, mean, similar = False, cand[0], None, None
    for it in range(min(max_iterations, len(rotations))):
        ref = rotations[it]
        ang = np.degrees((ref.inv() * rotations).magnitude())
        similar = np.where(ang < orientation_threshold)[0]
        if len(similar) >= min_required_matches:
            eqs = []
            for idx in similar:   # faiss_db.py:374-398 _find_symmetry_equivalent_orientation
                all_sym = quat_sym * rotations[idx]
                k = (ref.inv() * all_sym).magnitude().argmin()
                eqs.append(all_sym[k].as_euler("zxz", degrees=True))
            mean = R.from_euler("zxz", np.array(eqs), degrees=True).mean().as_euler("zxz", degrees=True)
            success, best = True, mean
            break
    return best, mean, success, similar
