"""On-device pattern ingest for the MI355X path (latice/data_module.py in the reference).

The reference converts one pattern at a time on CPU DataLoader workers
(`DPdataset.__getitem__`, data_module.py:125-133, through create_default_transform
:17-33: ToPILImage -> Grayscale -> CenterCrop -> ToTensor).  Here a whole batch of raw
patterns is copied to HBM once and transformed by one HIP launch
(`ebsdvae_ingest_patterns`, csrc/ingest.hip), so the training step and
build_dictionary are fed without a CPU stage per sample.

    ingest_patterns(raw (B, H0, W0) float64/float32, image_size) -> (B, 1, h, w) fp32 on device
    DPdataset(path, rot_angles_path, image_size)   .npy memmap + angle file (data_module.py:36-133)
        .batch(indices) -> (patterns on device, angles (B, 3) float64)
        .iter_batches(batch_size) -> device batches in order (pinned host staging)

There is no CPU fallback: the transform runs on the ROCm device or raises.
"""
from __future__ import annotations

import logging
from pathlib import Path

import numpy as np
import torch

from . import _native as N

logger = logging.getLogger(__name__)

_DTYPES = {torch.float64: 0, torch.float32: 1}


def ingest_patterns(raw, image_size=(128, 128), device="cuda", out: torch.Tensor | None = None):
    """Batched DPdataset transform on the device: raw (B, H0, W0) -> (B, 1, h, w) float32."""
    t = torch.as_tensor(raw)
    if t.dtype not in _DTYPES:
        t = t.to(torch.float64)   # data_module.py:132 casts every pattern to float64
    if t.ndim == 2:
        t = t.unsqueeze(0)
    if t.ndim != 3:
        raise ValueError(f"patterns must be (B, H, W), got {tuple(t.shape)}")
    t = t.to(device, non_blocking=True).contiguous()
    if not t.is_cuda:
        raise RuntimeError("ingest_patterns needs a ROCm device (no CPU fallback)")
    B, H0, W0 = t.shape
    h, w = image_size
    if out is None:
        out = torch.empty(B, 1, h, w, dtype=torch.float32, device=t.device)
    N.call("ebsdvae_ingest_patterns", t.data_ptr(), _DTYPES[t.dtype], B, H0, W0, h, w,
           N.ptr(out), N.stream(t.device))
    return out


def parse_rotation_angles(rot_angles_path) -> np.ndarray:
    """data_module.py:87-116: skip two header lines, whitespace-split "z1 x z2" rows."""
    with open(rot_angles_path) as f:
        lines = f.readlines()[2:]
    rows = [[a for a in line.strip().split(" ") if a] for line in lines]
    return np.asarray(rows, dtype=float).reshape(-1, 3)


class DPdataset:
    """data_module.py:36-133 with batched on-device transforms.  The pattern file is
    memory-mapped (the reference loads it whole, :70)."""

    def __init__(self, path, rot_angles_path, image_size=(128, 128), device="cuda") -> None:
        path = Path(path)
        try:
            self.ebsp_dataset = np.load(path, mmap_mode="r")
        except Exception as e:
            raise ValueError("Only .npy data files are supported.") from e
        if len(self.ebsp_dataset.shape) != 3:
            raise ValueError("The input dataset should be 3D.")
        self.rot_angles = parse_rotation_angles(rot_angles_path)
        self.image_size = tuple(image_size)
        self.device = torch.device(device)
        self._pinned = None

    def __len__(self) -> int:
        return self.ebsp_dataset.shape[0]

    def batch(self, indices):
        """(patterns (B, 1, h, w) fp32 on device, angles (B, 3) float64) for `indices`."""
        idx = np.asarray(indices, dtype=np.int64)
        raw = np.ascontiguousarray(self.ebsp_dataset[idx])
        if raw.dtype not in (np.float64, np.float32):
            raw = raw.astype(np.float64)
        host = torch.from_numpy(raw)
        if self._pinned is None or self._pinned.numel() < host.numel() or self._pinned.dtype != host.dtype:
            self._pinned = torch.empty(host.numel(), dtype=host.dtype).pin_memory()
        staged = self._pinned[: host.numel()].view(host.shape)
        staged.copy_(host)
        x = ingest_patterns(staged, self.image_size, self.device)
        return x, self.rot_angles[idx]

    def iter_batches(self, batch_size: int):
        for s in range(0, len(self), batch_size):
            yield self.batch(np.arange(s, min(s + batch_size, len(self))))
