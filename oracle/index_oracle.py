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
