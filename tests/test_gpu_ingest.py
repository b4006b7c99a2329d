"""On-device DPdataset transform (csrc/ingest.hip, latice.data_module) vs the restatement of
torchvision's ToPILImage -> Grayscale -> CenterCrop -> ToTensor (oracle/index_oracle.py):
bit-exact (integer uint8 path), over crop, odd-margin (round half to even) and pad cases."""
import numpy as np
import pytest
import torch

from latice import data_module as D
from oracle import index_oracle as IO

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("H0,W0,out", [(160, 160, (128, 128)), (129, 131, (128, 128)),
                                        (133, 135, (128, 128)), (100, 140, (128, 128)),
                                        (128, 128, (128, 128)), (64, 61, (64, 64))])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_ingest_matches_torchvision_restatement(cuda, H0, W0, out, dtype):
    rng = np.random.default_rng(H0 * 7 + W0)
    raw = rng.random((5, H0, W0)).astype(dtype)
    raw[0, :3, :3] = [[1.0, 0.0, -0.5], [1.5, np.nan, 0.999999], [1 / 255, 2 / 255, 0.5]]
    got = D.ingest_patterns(raw, out).cpu().numpy()
    assert np.array_equal(got, IO.ingest_patterns(raw, out))


def test_dpdataset_batches(cuda, tmp_path):
    rng = np.random.default_rng(2)
    raw = rng.random((10, 140, 140))
    np.save(tmp_path / "p.npy", raw)
    with open(tmp_path / "a.txt", "w") as f:
        f.write("eu\n10\n")
        for i in range(10):
            f.write(f"{i}.5  {2 * i} {3 * i}\n")
    ds = D.DPdataset(tmp_path / "p.npy", tmp_path / "a.txt", (128, 128))
    assert len(ds) == 10
    x, ang = ds.batch([3, 7])
    assert x.shape == (2, 1, 128, 128) and x.is_cuda
    assert np.array_equal(x.cpu().numpy(), IO.ingest_patterns(raw[[3, 7]]))
    assert np.allclose(ang, [[3.5, 6, 9], [7.5, 14, 21]])
    n = sum(b[0].shape[0] for b in ds.iter_batches(4))
    assert n == 10
