"""Call contracts of DiffractionPatternIndexer that the reference's own unit tests pin
(/root/reference/tests/index/test_dp_indexer.py), run against the drop-in
latice.index.dp_indexer with a mock model and a mock database (CPU only).

Pinned there and here:
  * __init__ calls model.eval() once and model.to(device) once (:117-119), falls back to
    CPU when CUDA is requested but unavailable (:121-133);
  * build_dictionary reads the cached-property dataloader once, extracts once and adds the
    vectors once (:135-174);
  * encode_pattern / encode_patterns_batch return numpy arrays for tensor and numpy input
    (:176-215);
  * index_pattern(s) forward top_n / orientation_threshold / batch_size to the database
    (:217-276);
  * _extract_latent_vectors_with_angles calls the model exactly ONCE per batch and keeps
    element [2] (:278-305) -- the reason the drop-in model's encoder-only fast path lives
    inside model(x) (deferred decoder) rather than replacing the call.
"""
import os
import sys
from unittest.mock import ANY, MagicMock, PropertyMock, patch

import numpy as np
import pytest
import torch

from latice.index.dp_indexer import DiffractionPatternIndexer, IndexerConfig
from latice.index.faiss_db import FaissLatentVectorDatabase, OrientationResult


def _orientation():
    return OrientationResult(query_vector=np.zeros(16), best_orientation=np.array([30.0, 45.0, 60.0]),
                             mean_orientation=np.array([31.0, 44.0, 61.0]),
                             candidate_orientations=np.zeros((5, 3)), distances=np.linspace(0.1, 0.5, 5),
                             success=True, similar_indices=np.arange(3))


@pytest.fixture
def model():
    m = MagicMock()
    m.eval.return_value = None
    m.return_value = (torch.randn(4, 16), torch.randn(4, 1, 128, 128), torch.randn(4, 16),
                      torch.randn(4, 16))
    return m


@pytest.fixture
def db():
    d = MagicMock(spec=FaissLatentVectorDatabase)
    d.find_best_orientation.return_value = _orientation()
    d.find_best_orientations_batch.return_value = [_orientation()] * 3
    return d


@pytest.fixture
def config(tmp_path):
    np.save(tmp_path / "patterns.npy", np.random.default_rng(0).random((10, 128, 128)))
    np.save(tmp_path / "angles.npy", np.random.default_rng(1).random((10, 3)) * 360)
    return IndexerConfig(pattern_path=tmp_path / "patterns.npy", angles_path=tmp_path / "angles.npy",
                         batch_size=2, device="cpu", latent_dim=16, image_size=(128, 128), top_n=5,
                         orientation_threshold=2.0)


def _indexer(model, db, config):
    with patch.object(DiffractionPatternIndexer, "build_dictionary"):
        return DiffractionPatternIndexer(model, db, config)


def test_init_prepares_model_once(model, db, config):
    ix = _indexer(model, db, config)
    assert ix.model is model and ix.db is db and ix.config is config
    assert str(ix.device) == "cpu"
    model.eval.assert_called_once()
    model.to.assert_called_once_with(torch.device("cpu"))


def test_init_falls_back_to_cpu(model, db, config):
    config.device = "cuda"
    with patch("torch.cuda.is_available", return_value=False):
        ix = _indexer(model, db, config)
    assert str(ix.device) == "cpu"


def test_build_dictionary_flow(model, db, config):
    loader = MagicMock()
    lat, ori = np.random.rand(10, 16), np.random.rand(10, 3)
    with patch.object(DiffractionPatternIndexer, "_create_dataloader", new_callable=PropertyMock,
                      return_value=loader) as mk, \
            patch.object(DiffractionPatternIndexer, "_extract_latent_vectors_with_angles",
                         return_value=(lat, ori)) as ex, \
            patch.object(DiffractionPatternIndexer, "__init__", return_value=None):
        ix = DiffractionPatternIndexer()
        ix.model, ix.db, ix.config, ix.device = model, db, config, torch.device("cpu")
        ix.build_dictionary()
    mk.assert_called_once()
    ex.assert_called_once_with(loader)
    db.add_vectors.assert_called_once_with(lat, ori)


def test_encode_pattern_returns_numpy(model, db, config):
    ix = _indexer(model, db, config)
    assert isinstance(ix.encode_pattern(torch.rand(128, 128)), np.ndarray)
    with patch("latice.index.dp_indexer.create_default_transform", return_value=lambda a: torch.tensor(a)):
        assert isinstance(ix.encode_pattern(np.random.rand(128, 128)), np.ndarray)


def test_encode_patterns_batch_returns_numpy(model, db, config):
    ix = _indexer(model, db, config)
    assert isinstance(ix.encode_patterns_batch(torch.rand(3, 128, 128)), np.ndarray)
    with patch("latice.index.dp_indexer.create_default_transform",
               return_value=lambda a: torch.tensor(a).unsqueeze(1)):
        assert isinstance(ix.encode_patterns_batch(np.random.rand(3, 128, 128)), np.ndarray)


def test_index_pattern_forwards_thresholds(model, db, config):
    with patch.object(DiffractionPatternIndexer, "encode_pattern", return_value=np.random.rand(16)):
        ix = _indexer(model, db, config)
        ix.index_pattern(torch.rand(128, 128))
        db.find_best_orientation.assert_called_with(ANY, top_n=config.top_n,
                                                    orientation_threshold=config.orientation_threshold)
        ix.index_pattern(torch.rand(128, 128), top_n=10, orientation_threshold=1.5)
        db.find_best_orientation.assert_called_with(ANY, top_n=10, orientation_threshold=1.5)


def test_index_patterns_batch_forwards_batch_size(model, db, config):
    with patch.object(DiffractionPatternIndexer, "encode_patterns_batch", return_value=np.random.rand(3, 16)):
        ix = _indexer(model, db, config)
        ix.index_patterns_batch(torch.rand(3, 128, 128))
        db.find_best_orientations_batch.assert_called_once()
        ix.index_patterns_batch(torch.rand(3, 128, 128), top_n=10, orientation_threshold=1.5)
        db.find_best_orientations_batch.assert_called_with(ANY, batch_size=config.batch_size, top_n=10,
                                                           orientation_threshold=1.5)


def test_extract_calls_model_once_per_batch(model, db, config):
    loader = MagicMock()
    loader.__iter__.return_value = iter([(torch.rand(2, 1, 128, 128), torch.rand(2, 3)),
                                         (torch.rand(1, 1, 128, 128), torch.rand(1, 3))])
    loader.__len__.return_value = 2
    mu = torch.randn(1, 16)
    model.return_value = (torch.randn(1, 1, 128, 128), None, mu, torch.randn(1, 16))
    ix = _indexer(model, db, config)
    lat, ori = ix._extract_latent_vectors_with_angles(loader)
    assert isinstance(lat, np.ndarray) and isinstance(ori, np.ndarray)
    assert model.call_count == 2
    assert np.array_equal(lat[0], mu.numpy()[0])   # element [2] of the model's output
    assert ori.shape == (3, 3)


def test_reference_checkout_fills_in_unreplaced_modules(tmp_path):
    """LATICE_REFERENCE_ROOT: modules the drop-in does not replace resolve from a reference
    checkout; the drop-in's own modules keep precedence (run in a subprocess so the
    environment variable is seen at package import)."""
    import subprocess
    ref = tmp_path / "ref"
    (ref / "latice" / "utils").mkdir(parents=True)
    (ref / "latice" / "index").mkdir(parents=True)
    (ref / "latice" / "__init__.py").write_text("")
    (ref / "latice" / "utils" / "__init__.py").write_text("")
    (ref / "latice" / "utils" / "constants.py").write_text("FROM_REFERENCE = True\n")
    (ref / "latice" / "index" / "chroma_db.py").write_text("FROM_REFERENCE = True\n")
    (ref / "latice" / "model.py").write_text("raise ImportError('reference model must not load')\n")
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ebsd-vae_amd")
    code = ("import latice.utils.constants as c, latice.index.chroma_db as d, latice.model as m;"
            "assert c.FROM_REFERENCE and d.FROM_REFERENCE;"
            "assert m.__file__.startswith(%r)" % pkg)
    env = dict(os.environ, LATICE_REFERENCE_ROOT=str(ref), PYTHONPATH=pkg)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
