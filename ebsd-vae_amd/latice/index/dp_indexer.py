"""Drop-in `latice.index.dp_indexer` (reference: latice/index/dp_indexer.py) on the MI355X
path: same `IndexerConfig` and `DiffractionPatternIndexer` API and call contracts.

* `build_dictionary` (:92-111) -> `_create_dataloader` (:234-252, the drop-in DPDataModule:
  device batches from one transform launch each) -> `_extract_latent_vectors_with_angles`
  (:254-297), which calls `self.model(data)` exactly once per batch and keeps `mu`, as the
  reference's tests pin (tests/index/test_dp_indexer.py:117-119, :305).  With the drop-in
  model that call runs the encoder and the heads only: its eval/no-grad forward defers the
  decoder (latice.model, latice.deferred).
* The default database is the HBM-resident `FaissLatentVectorDatabase` (exact cosine top-k +
  batched orientation consensus as HIP kernels); the reference defaults to a Chroma HNSW
  collection (chromadb is a third-party service, out of scope).  Any object with
  add_vectors / find_best_orientation / find_best_orientations_batch can be passed as `db`.
* encode_patterns_batch transforms a numpy stack in ONE launch when the transform is the
  default one (the reference loops per pattern, :149-163).
"""
from __future__ import annotations

import logging
from functools import cached_property
from pathlib import Path
from typing import Literal

import numpy as np
import torch
from pydantic.dataclasses import dataclass

from latice.data_module import DPDataModule, PatternTransform, create_default_transform
from latice.index.faiss_db import (FaissLatentVectorDatabase, FaissLatentVectorDatabaseConfig,
                                   OrientationResult)
from latice.model import VariationalAutoEncoder

logger = logging.getLogger(__name__)

__all__ = ["IndexerConfig", "DiffractionPatternIndexer", "OrientationResult"]


@dataclass
class IndexerConfig:
    """dp_indexer.py:26-48 (identical fields and defaults)."""

    pattern_path: Path
    angles_path: Path
    batch_size: int = 64
    device: Literal["cuda", "cpu", "mps"] = "cpu"
    latent_dim: int = 16
    random_seed: int = 42
    image_size: tuple[int, int] = (128, 128)
    top_n: int = 20
    orientation_threshold: float = 3.0


def _default_db(dimension: int, device: torch.device):
    """The reference's default store is `ChromaLatentVectorDatabase(dimension=...)`
    (dp_indexer.py:73-77).  It is used when `latice.index.chroma_db` resolves (a reference
    checkout on LATICE_REFERENCE_ROOT and chromadb installed); otherwise the HBM-resident
    exact inner-product store `FaissLatentVectorDatabase` takes its place, with a warning
    (same add / query API, exact instead of HNSW search)."""
    try:
        from latice.index.chroma_db import ChromaLatentVectorDatabase
    except Exception as e:  # noqa: BLE001 - chromadb or the module absent
        logger.warning("ChromaLatentVectorDatabase is not available (%s: %s); using the "
                       "HBM-resident exact FaissLatentVectorDatabase as the default store",
                       type(e).__name__, e)
        return FaissLatentVectorDatabase(
            FaissLatentVectorDatabaseConfig(dimension=dimension, device=str(device)))
    return ChromaLatentVectorDatabase(dimension=dimension)


class DiffractionPatternIndexer:
    """dp_indexer.py:51-297."""

    def __init__(self, model: VariationalAutoEncoder, db=None, config: IndexerConfig | None = None) -> None:
        self.config = config if config is not None else IndexerConfig()
        np.random.seed(self.config.random_seed)
        torch.manual_seed(self.config.random_seed)
        self.device = torch.device(self.config.device)
        if self.config.device == "cuda" and not torch.cuda.is_available():
            logger.warning("CUDA not available, falling back to CPU")
            self.device = torch.device("cpu")
        logger.info(f"Using device: {self.device}")
        if self.device.type == "cpu" and isinstance(model, VariationalAutoEncoder):
            # the drop-in model has no CPU path: IndexerConfig's default device "cpu" would
            # only fail later, deep inside the first encode
            if not torch.cuda.is_available():
                raise RuntimeError("DiffractionPatternIndexer: the MI355X VAE needs a ROCm device "
                                   "(config.device='cpu' and no GPU is visible; no CPU fallback)")
            logger.warning("config.device='cpu': the drop-in VAE runs on the ROCm device; using "
                           "cuda:%d", torch.cuda.current_device())
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.db = db if db is not None else _default_db(self.config.latent_dim, self.device)
        self.model = model
        self.model.eval()
        self.model.to(self.device)

    def build_dictionary(self) -> None:
        """dp_indexer.py:92-111: latent vectors of every pattern -> the database."""
        data_module = self._create_dataloader
        logger.info(f"Generating latent vectors from patterns in {self.config.pattern_path}")
        latent_vectors, orientations = self._extract_latent_vectors_with_angles(data_module)
        logger.info(f"Adding {len(latent_vectors)} vectors to database")
        self.db.add_vectors(latent_vectors, orientations)

    def encode_pattern(self, pattern) -> np.ndarray:
        """dp_indexer.py:113-136."""
        transform = create_default_transform(self.config.image_size)
        if isinstance(pattern, np.ndarray):
            pattern = transform(pattern)
        if pattern.dim() == 2:
            pattern = pattern.unsqueeze(0)
        if pattern.dim() == 3:
            pattern = pattern.unsqueeze(0)
        pattern = pattern.to(self.device)
        with torch.no_grad():
            _, _, mu, _ = self.model(pattern)
        return mu.cpu().numpy().squeeze()

    def encode_patterns_batch(self, patterns) -> np.ndarray:
        """dp_indexer.py:138-186."""
        transform = create_default_transform(self.config.image_size)
        if isinstance(patterns, np.ndarray):
            if patterns.ndim == 2:
                patterns = transform(patterns).unsqueeze(0)
            elif patterns.ndim == 3:
                if isinstance(transform, PatternTransform):
                    patterns = transform.batch(patterns)   # one launch for the whole stack
                else:
                    patterns = torch.stack([transform(patterns[i]) for i in range(patterns.shape[0])])
        else:
            if patterns.dim() == 2:
                patterns = patterns.unsqueeze(0).unsqueeze(0)
            elif patterns.dim() == 3:
                patterns = patterns.unsqueeze(1)
        assert patterns.dim() == 4, f"Expected 4D tensor, got {patterns.dim()}D"
        patterns = patterns.to(self.device)
        batch_size = self.config.batch_size
        latent_vectors = []
        with torch.no_grad():
            for i in range(0, patterns.shape[0], batch_size):
                _, _, mu, _ = self.model(patterns[i:i + batch_size])
                latent_vectors.append(mu.cpu().numpy())
        return np.vstack(latent_vectors)

    def index_pattern(self, pattern, top_n: int | None = None,
                      orientation_threshold: float | None = None) -> OrientationResult:
        """dp_indexer.py:188-214."""
        top_n = top_n or self.config.top_n
        orientation_threshold = orientation_threshold or self.config.orientation_threshold
        latent_vector = self.encode_pattern(pattern)
        return self.db.find_best_orientation(latent_vector, top_n=top_n,
                                             orientation_threshold=orientation_threshold)

    def index_patterns_batch(self, patterns, **kwargs):
        """dp_indexer.py:216-232."""
        latent_vectors = self.encode_patterns_batch(patterns)
        return self.db.find_best_orientations_batch(latent_vectors, batch_size=self.config.batch_size,
                                                    **kwargs)

    @cached_property
    def _create_dataloader(self):
        """dp_indexer.py:234-252."""
        datamodule = DPDataModule(path=self.config.pattern_path,
                                  rot_angles_path=self.config.angles_path,
                                  image_size=self.config.image_size,
                                  batch_size=self.config.batch_size)
        datamodule.setup("test")
        return datamodule.test_dataloader()

    def _extract_latent_vectors_with_angles(self, data_loader):
        """dp_indexer.py:254-297: one model call per batch, mu kept (a rich progress bar as
        in the reference when rich is importable)."""
        latent_vectors, orientations = [], []
        try:
            from rich.progress import (BarColumn, Progress, SpinnerColumn, TextColumn,
                                       TimeElapsedColumn)
            progress = Progress(SpinnerColumn(), TextColumn("[progress.description]{task.description}"),
                                BarColumn(), TextColumn("[progress.percentage]{task.percentage:>3.0f}%"),
                                TimeElapsedColumn())
        except Exception:  # noqa: BLE001
            progress = None
        ctx = progress if progress is not None else _NullProgress()
        with ctx:
            task = ctx.add_task("[cyan]Processing patterns...", total=len(data_loader))
            with torch.no_grad():
                for batch in data_loader:
                    data, angles = batch
                    data = data.to(self.device)
                    _, _, mu, _ = self.model(data)
                    latent_vectors.append(mu.cpu().numpy())
                    orientations.append(np.asarray(angles))
                    ctx.update(task, advance=1)
        return np.concatenate(latent_vectors, axis=0), np.concatenate(orientations, axis=0)


class _NullProgress:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def add_task(self, *a, **k):
        return 0

    def update(self, *a, **k):
        return None
