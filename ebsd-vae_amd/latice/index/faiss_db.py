"""Drop-in for latice/index/faiss_db.py (FaissLatentVectorDatabase) on the MI355X path.

The reference keeps L2-normalised latent vectors in a faiss-cpu 1.10 `IndexFlatIP`
(exhaustive inner product = cosine similarity, faiss_db.py:126-139) and answers
`query_similar` one query at a time (:216-256).  Here the normalised dictionary lives in HBM
as an N x D fp32 tensor and queries run as batched HIP launches (csrc/search.hip):

    ebsdvae_l2_normalize_rows   faiss_db.py:107-111 (norm 0 -> 1)
    ebsdvae_cosine_topk         IndexFlatIP.search: k best by score, ties to the lower row
    ebsdvae_orient_consensus    find_best_orientation (:258-398), all queries in one launch

There is no CPU or faiss fallback: the dictionary must sit on a ROCm device.  Persistence
is one .npz with the normalised `latents` and the `orientations` (the reference pickles a
serialised faiss index into the same file, faiss_db.py:426-445; that format needs faiss).
"""
from __future__ import annotations

import logging
from dataclasses import dataclass
from pathlib import Path

import numpy as np
import torch

from .. import _native as N

logger = logging.getLogger(__name__)

MAX_K = 64


@dataclass
class FaissLatentVectorDatabaseConfig:
    """faiss_db.py:35-46 (+ the device the dictionary lives on)."""
    npz_path: str = "faiss_index.npz"
    dimension: int = 16
    device: str = "cuda"


@dataclass
class OrientationResult:
    """faiss_db.py:49-89 (identical fields)."""
    query_vector: np.ndarray
    best_orientation: np.ndarray
    candidate_orientations: np.ndarray
    distances: np.ndarray
    mean_orientation: np.ndarray | None = None
    success: bool = True
    similar_indices: np.ndarray | None = None

    def get_top_n_orientations(self, n: int = 5) -> np.ndarray:
        """faiss_db.py:72-89 (sorts by ascending distance, as the reference does)."""
        if self.distances is None or len(self.distances) == 0:
            return self.candidate_orientations[: min(n, len(self.candidate_orientations))]
        order = np.argsort(self.distances)
        return self.candidate_orientations[order[: min(n, len(order))]]


def _as_device_f32(x, device) -> torch.Tensor:
    t = torch.as_tensor(x)
    return t.to(device=device, dtype=torch.float32).contiguous()


def l2_normalize(x: torch.Tensor) -> torch.Tensor:
    """Row-wise v / ||v|| on the device (faiss_db.py:107-111)."""
    if not x.is_cuda:
        raise RuntimeError("l2_normalize needs a ROCm device tensor (no CPU fallback)")
    x = x.to(torch.float32).contiguous()
    y = torch.empty_like(x)
    N.call("ebsdvae_l2_normalize_rows", x.data_ptr(), y.data_ptr(), x.shape[0], x.shape[1],
           N.stream(x.device))
    return y


def cosine_topk(db: torch.Tensor, queries: torch.Tensor, k: int):
    """Exact top-k of <q, db_i> over normalised rows; (scores (Q,k) fp32, idx (Q,k) int64),
    best first, ties to the lower row index."""
    if not (db.is_cuda and queries.is_cuda):
        raise RuntimeError("cosine_topk needs ROCm device tensors (no CPU fallback)")
    n, d = db.shape
    q = queries.reshape(-1, d).contiguous()
    Q = q.shape[0]
    scores = torch.empty(Q, k, dtype=torch.float32, device=db.device)
    idx = torch.empty(Q, k, dtype=torch.int64, device=db.device)
    nbytes = N.call("ebsdvae_cosine_topk_work", n, Q, d, k)
    work = torch.empty(max(nbytes, 8), dtype=torch.uint8, device=db.device)
    N.call("ebsdvae_cosine_topk", db.data_ptr(), n, q.data_ptr(), Q, d, k, scores.data_ptr(),
           idx.data_ptr(), work.data_ptr(), N.stream(db.device))
    return scores, idx


class FaissLatentVectorDatabase:
    """faiss_db.py:92-496 with an HBM-resident dictionary and HIP search."""

    def __init__(self, config: FaissLatentVectorDatabaseConfig | None = None) -> None:
        self.config = config if config is not None else FaissLatentVectorDatabaseConfig()
        self.dimension = self.config.dimension
        self.npz_path = Path(self.config.npz_path)
        self.device = torch.device(self.config.device)
        self._reset()
        if self.npz_path.exists():
            self.load()
        else:
            logger.info(f"No existing index found at {self.npz_path}. Creating a new one.")

    # ------------------------------------------------------------------ storage
    # Capacity-backed (amortised doubling), so appending batch after batch -- the
    # build_dictionary pattern -- costs O(N) copies overall, not O(N^2).
    def _reset(self, capacity: int = 0) -> None:
        self._n = 0
        self._cap_db = torch.empty(capacity, self.dimension, dtype=torch.float32, device=self.device)
        self._cap_ori = np.empty((capacity, 3), dtype=np.float64)
        self._cap_ori_dev = torch.empty(capacity, 3, dtype=torch.float64, device=self.device)

    def reserve(self, capacity: int) -> None:
        """Pre-size the dictionary for `capacity` rows (optional)."""
        if capacity <= self._cap_db.shape[0]:
            return
        db, ori, ord_ = self._cap_db, self._cap_ori, self._cap_ori_dev
        n = self._n
        self._cap_db = torch.empty(capacity, self.dimension, dtype=torch.float32, device=self.device)
        self._cap_ori = np.empty((capacity, 3), dtype=np.float64)
        self._cap_ori_dev = torch.empty(capacity, 3, dtype=torch.float64, device=self.device)
        self._cap_db[:n].copy_(db[:n])
        self._cap_ori[:n] = ori[:n]
        self._cap_ori_dev[:n].copy_(ord_[:n])

    @property
    def _db(self) -> torch.Tensor:
        return self._cap_db[: self._n]

    @property
    def _orientations(self) -> np.ndarray:
        return self._cap_ori[: self._n]

    @property
    def _ori_dev(self) -> torch.Tensor:
        return self._cap_ori_dev[: self._n]

    def _append(self, lv: torch.Tensor, ori: np.ndarray, ori_dev: torch.Tensor | None = None) -> None:
        n, m = self._n, lv.shape[0]
        if n + m > self._cap_db.shape[0]:
            self.reserve(max(n + m, 2 * self._cap_db.shape[0], 1024))
        self._cap_db[n:n + m].copy_(lv)
        self._cap_ori[n:n + m] = ori
        self._cap_ori_dev[n:n + m].copy_(ori_dev if ori_dev is not None else torch.from_numpy(ori))
        self._n = n + m

    # ------------------------------------------------------------------ population
    def _validate_vectors(self, latent_vectors, orientations) -> None:
        """faiss_db.py:141-158."""
        if len(latent_vectors) != len(orientations):
            raise ValueError("Number of latent vectors and orientations must match")
        if latent_vectors.shape[1] != self.dimension:
            raise ValueError(f"Expected latent vectors of dimension {self.dimension}, "
                             f"got {latent_vectors.shape[1]}")
        if orientations.shape[1] != 3:
            raise ValueError(f"Expected orientations of shape (n, 3), got {orientations.shape}")

    def add_vectors(self, latent_vectors, orientations) -> None:
        """faiss_db.py:160-189: cast to fp32, L2-normalise, append (numpy or device tensors;
        device tensors from `encode_mu` never leave HBM)."""
        orientations = np.asarray(orientations, dtype=np.float64)
        if orientations.ndim == 1:
            orientations = orientations.reshape(-1, 3)
        lv = _as_device_f32(latent_vectors, self.device)
        if lv.ndim != 2:
            raise ValueError(f"latent vectors must be 2-D, got shape {tuple(lv.shape)}")
        lv = l2_normalize(lv) if lv.shape[0] else lv
        self._validate_vectors(lv, orientations)
        self._append(lv, orientations)
        logger.info(f"Added {lv.shape[0]} vectors. Index total: {self.get_count()}")

    def create_from_files(self, latent_file_path, angles_file_path) -> None:
        """faiss_db.py:191-214."""
        lv = np.load(Path(latent_file_path)).astype(np.float32)
        ori = np.load(Path(angles_file_path))
        self.add_vectors(lv, ori)
        self.save()

    # ------------------------------------------------------------------ queries
    def query_similar_batch(self, query_vectors, n_results: int = 20):
        """Batched query_similar: (distances (Q,k) fp32, indices (Q,k) int64) as numpy, the
        GPU search running once for all Q queries."""
        count = self.get_count()
        if count == 0:
            logger.warning("Querying an empty index.")
            return np.empty((0, 0), np.float32), np.empty((0, 0), np.int64)
        if count < n_results:
            logger.warning(f"Requested {n_results} results, but index only contains {count} "
                           "vectors. Returning all.")
            n_results = count
        if n_results > MAX_K:
            raise ValueError(f"n_results={n_results} > {MAX_K} (GPU top-k limit)")
        q = _as_device_f32(query_vectors, self.device)
        if q.ndim == 1:
            q = q.reshape(1, -1)
        if q.shape[1] != self.dimension:
            raise ValueError(f"Expected query vector of dimension {self.dimension}, got {q.shape[1]}")
        s, i = cosine_topk(self._db, l2_normalize(q), n_results)
        return s.cpu().numpy(), i.cpu().numpy()

    def query_similar(self, query_vector, n_results: int = 20):
        """faiss_db.py:216-256: distances (cosine similarity) and indices of one query."""
        d, i = self.query_similar_batch(query_vector, n_results)
        if d.size == 0:
            return np.array([]), np.array([])
        return d[0], i[0]

    # ------------------------------------------------------------------ orientation consensus
    def find_best_orientations_batch(self, query_vectors, batch_size: int = 32, top_n: int = 20,
                                     orientation_threshold: float = 1.0,
                                     min_required_matches: int = 18,
                                     max_iterations: int = 3) -> list[OrientationResult]:
        """faiss_db.py:400-438 (which loops find_best_orientation per vector): here ONE
        cosine top-k launch and ONE consensus launch serve every query (batch_size only
        bounds the launch size)."""
        qv = np.asarray(query_vectors.detach().cpu() if torch.is_tensor(query_vectors) else query_vectors)
        qv = qv.reshape(-1, self.dimension)
        count = self.get_count()
        if count == 0:
            logger.warning("No similar vectors found for query.")
            return [OrientationResult(query_vector=v.squeeze(), best_orientation=np.full(3, np.nan),
                                      candidate_orientations=np.array([]), distances=np.array([]),
                                      mean_orientation=None, success=False, similar_indices=None)
                    for v in qv]
        k = min(top_n, count)
        if k > MAX_K:
            raise ValueError(f"top_n={top_n} > {MAX_K} (GPU top-k limit)")
        out = []
        step = max(int(batch_size), 1) * 1024   # queries per launch pair
        for s0 in range(0, len(qv), step):
            q = _as_device_f32(qv[s0:s0 + step], self.device)
            scores, idx = cosine_topk(self._db, l2_normalize(q), k)
            Q = q.shape[0]
            best = torch.empty(Q, 3, dtype=torch.float64, device=self.device)
            mean = torch.empty(Q, 3, dtype=torch.float64, device=self.device)
            ok = torch.empty(Q, dtype=torch.int32, device=self.device)
            mask = torch.empty(Q, dtype=torch.int64, device=self.device)
            N.call("ebsdvae_orient_consensus", self._ori_dev.data_ptr(), idx.data_ptr(), Q, k,
                   float(orientation_threshold), int(min_required_matches), int(max_iterations),
                   best.data_ptr(), mean.data_ptr(), ok.data_ptr(), mask.data_ptr(),
                   N.stream(self.device))
            scores, idx = scores.cpu().numpy(), idx.cpu().numpy()
            best, mean = best.cpu().numpy(), mean.cpu().numpy()
            ok, mask = ok.cpu().numpy(), mask.cpu().numpy().view(np.uint64)
            iters = min(max_iterations, k)
            bits = ((mask[:, None] >> np.arange(k, dtype=np.uint64)) & np.uint64(1)).astype(bool)
            cands = self._orientations[idx]                   # (Q, k, 3)
            lanes = np.arange(k, dtype=np.int64)
            n_fail = int(Q - ok.sum())
            if n_fail:
                logger.warning(f"Failed to find consensus orientation for {n_fail} of {Q} queries "
                               f"after {iters} iterations; their best guess is the closest match")
            for j in range(Q):
                sim = lanes[bits[j]] if iters > 0 else None
                succ = bool(ok[j])
                out.append(OrientationResult(
                    query_vector=qv[s0 + j].squeeze().astype(np.float64),
                    best_orientation=best[j], mean_orientation=mean[j] if succ else None,
                    candidate_orientations=cands[j], distances=scores[j],
                    success=succ, similar_indices=sim))
        return out

    def find_best_orientation(self, query_vector, top_n: int = 20,
                              orientation_threshold: float = 1.0, min_required_matches: int = 18,
                              max_iterations: int = 3) -> OrientationResult:
        """faiss_db.py:258-372 for one query (runs the batched kernels with Q = 1)."""
        return self.find_best_orientations_batch(
            np.asarray(query_vector).reshape(1, -1), top_n=top_n,
            orientation_threshold=orientation_threshold,
            min_required_matches=min_required_matches, max_iterations=max_iterations)[0]

    # ------------------------------------------------------------------ bookkeeping
    def get_count(self) -> int:
        return int(self._n)

    @property
    def orientations(self) -> np.ndarray:
        return self._orientations

    def save(self) -> None:
        """One .npz: normalised latents + orientations (faiss_db.py:426-445 stores a faiss
        blob instead)."""
        np.savez_compressed(str(self.npz_path.with_suffix(".npz")),
                            latents=self._db.cpu().numpy(), orientations=self._orientations)
        logger.info(f"Saved index and metadata to {self.npz_path.with_suffix('.npz')}")

    def load(self) -> None:
        """faiss_db.py:447-466 for the .npz this class writes (no pickles)."""
        path = self.npz_path.with_suffix(".npz")
        if not path.exists():
            raise FileNotFoundError("NPZ file missing.")
        with np.load(str(path), allow_pickle=False) as data:
            if "latents" not in data:
                raise ValueError(f"{path} has no 'latents' array (a faiss-serialised index "
                                 "needs faiss to read; re-create it with add_vectors)")
            lv = data["latents"].astype(np.float32)
            ori = data["orientations"].astype(np.float64).reshape(-1, 3)
        self.dimension = lv.shape[1]
        self._reset(lv.shape[0])
        self._append(torch.from_numpy(lv).to(self.device), ori)

    def delete_persistence(self) -> None:
        """faiss_db.py:468-496."""
        if self.npz_path.exists():
            self.npz_path.unlink()
            self._reset()
