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


# ----------------------------------------------------------------------------- ingest
def _py_round_half_even(x: float) -> int:
    return int(round(x))   # Python's round: ties to even, as torchvision's center_crop uses


def ingest_patterns(raw: np.ndarray, image_size=(128, 128)) -> np.ndarray:
    """latice/data_module.py:17-33,125-133: float64 cast, torchvision ToPILImage on a float
    ndarray ((x * 255).astype(uint8), clamped here to [0, 255] -- numpy's out-of-range cast is
    platform-defined), Grayscale (identity on "L"), CenterCrop (zero pad ((c-s)//2,
    (c-s+1)//2) when too small, else offset round((s-c)/2)), ToTensor (/255 in float32).
    torchvision 0.21 is not installed here: this restates its published algorithm (parity with
    torchvision itself unpinned)."""
    x = np.asarray(raw, dtype=np.float64)
    if x.ndim == 2:
        x = x[None]
    B, H0, W0 = x.shape
    u8 = np.clip(np.nan_to_num(x * 255.0, nan=0.0), 0, 255).astype(np.uint8)
    h, w = image_size
    out = np.zeros((B, 1, h, w), np.float32)

    def axis(size, crop):
        if crop > size:
            return -((crop - size) // 2)
        return _py_round_half_even((size - crop) / 2.0)

    top, left = axis(H0, h), axis(W0, w)
    for y in range(h):
        sy = y + top
        if not 0 <= sy < H0:
            continue
        xs = np.arange(w) + left
        ok = (xs >= 0) & (xs < W0)
        out[:, 0, y, ok] = u8[:, sy, xs[ok]].astype(np.float32) / np.float32(255.0)
    return out
