"""Drop-in `latice.data_module` (reference: latice/data_module.py) with the pattern transform
on the MI355X.

The reference converts one pattern at a time on CPU DataLoader workers
(`DPdataset.__getitem__`, data_module.py:122-133, through `create_default_transform`
:17-33: ToPILImage -> Grayscale -> CenterCrop -> ToTensor).  Here the same transform runs as
one HIP launch over a whole batch (`ebsdvae_ingest_patterns`, csrc/ingest.hip: float -> x255
-> uint8 cast, centre crop / zero pad, /255), fed from a memory-mapped .npy through pinned
host buffers that a background thread fills while the GPU works.

Same public names, constructor arguments and behaviour as the reference:

    create_default_transform(image_size)  -> callable: one (H, W) pattern -> (1, h, w) fp32
    DPdataset(path, rot_angles_path, image_size, transform)   data_module.py:36-133
    DPDataModule(path, rot_angles_path, image_size, val_data_ratio, batch_size, n_cpu,
                 seed, transform)                             data_module.py:136-261
        .setup(stage)   random_split(seed) for "fit", the whole set for "test" (:194-213)
        .train_dataloader() / .val_dataloader() / .test_dataloader()
            iterables of (patterns (B, 1, h, w) fp32 ON THE DEVICE, angles (B, 3) float64)
            with len() = number of batches, as torch DataLoaders of the reference's
            collated batches (callers' `data.to(device)` is then a no-op).

Lightning is optional: DPDataModule subclasses `pl.LightningDataModule` when
pytorch_lightning is importable.  There is no CPU fallback: the transform runs on the ROCm
device or raises.  A user-supplied `transform` (any callable of the reference's kind) is
honoured per pattern, exactly as the reference applies it.
"""
from __future__ import annotations

import logging
import math
import threading
from pathlib import Path

import numpy as np
import torch
from torch.utils.data import random_split

from . import _native as N

try:  # pragma: no cover - depends on the environment
    import pytorch_lightning as pl
    _DMBase = pl.LightningDataModule
except Exception:  # noqa: BLE001
    pl = None
    _DMBase = object

logger = logging.getLogger(__name__)

_DTYPES = {torch.float64: 0, torch.float32: 1}


def _default_device() -> torch.device:
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device("cuda")


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


class PatternTransform:
    """What `create_default_transform(image_size)` returns (data_module.py:17-33): called on
    one pattern -- an (H, W) or (1, H, W) array or tensor -- it returns the (1, h, w) float32
    tensor torchvision's ToPILImage -> Grayscale -> CenterCrop -> ToTensor would, computed on
    the device.  `.batch(raw)` transforms a whole (B, H, W) stack in one launch."""

    def __init__(self, image_size, device=None):
        self.image_size = tuple(image_size) if not isinstance(image_size, int) else (image_size,) * 2
        self.device = torch.device(device) if device is not None else None

    def _dev(self):
        return self.device if self.device is not None else _default_device()

    def __call__(self, pattern):
        t = torch.as_tensor(pattern)
        if t.ndim == 3 and t.shape[0] == 1:
            t = t[0]
        if t.ndim != 2:
            raise ValueError(f"expected one (H, W) pattern, got {tuple(t.shape)}")
        return ingest_patterns(t, self.image_size, self._dev())[0]

    def batch(self, raw):
        return ingest_patterns(raw, self.image_size, self._dev())

    def __repr__(self):
        return f"PatternTransform(image_size={self.image_size}, device={self.device})"


def create_default_transform(image_size: tuple[int, int]) -> PatternTransform:
    """data_module.py:17-33 (ToPILImage -> Grayscale -> CenterCrop(image_size) -> ToTensor)."""
    return PatternTransform(image_size)


def parse_rotation_angles(rot_angles_path) -> np.ndarray:
    """data_module.py:87-116: skip two header lines, whitespace-split "z1 x z2" rows."""
    try:
        with open(rot_angles_path) as f:
            lines = f.readlines()[2:]
        rows = [[a for a in line.strip().split(" ") if a] for line in lines]
        return np.asarray(rows, dtype=float).reshape(-1, 3)
    except FileNotFoundError:
        logger.error(f"Rotation angles file not found: {rot_angles_path}")
        raise
    except Exception as e:  # noqa: BLE001
        raise ValueError(f"Failed to parse rotation angles file: {e}") from e


class DPdataset:
    """data_module.py:36-133.  The pattern file is memory-mapped (the reference loads it
    whole, :70); `rot_angles` is the same pandas DataFrame (z1, x, z2).  Indexing returns
    (transform(pattern) (1, h, w), angles (3,) float64) like the reference; `batch(indices)`
    returns a whole device batch from one pinned copy and one transform launch."""

    def __init__(self, path, rot_angles_path, image_size=(128, 128), transform=None,
                 device=None) -> None:
        path = Path(path)
        try:
            self.ebsp_dataset = np.load(path, mmap_mode="r")
            logger.info(f"Loaded diffraction pattern data from {path}")
        except Exception as e:  # noqa: BLE001
            raise ValueError("Only .npy data files are supported.") from e
        if len(self.ebsp_dataset.shape) != 3:
            raise ValueError("The input dataset should be 3D.")
        self._angles = parse_rotation_angles(rot_angles_path)
        self.image_size = tuple(image_size)
        self.transform = transform or create_default_transform(self.image_size)
        self.device = torch.device(device) if device is not None else None
        self._pinned = None
        self._pinned_free = None   # HIP event: the last device copy out of _pinned finished

    @property
    def rot_angles(self):
        import pandas as pd
        return pd.DataFrame(self._angles, columns=["z1", "x", "z2"])

    def __len__(self) -> int:
        return self.ebsp_dataset.shape[0]

    def __getitem__(self, idx: int):
        dp = np.asarray(self.ebsp_dataset[idx]).astype(np.float64)
        return self.transform(dp), self._angles[idx].copy()

    def _dev(self):
        return self.device if self.device is not None else _default_device()

    def load_raw(self, indices, out: torch.Tensor | None = None) -> torch.Tensor:
        """Raw patterns of `indices` (sorted runs read straight from the memmap) copied into
        the host tensor `out` (pinned) or a new one."""
        idx = np.asarray(indices, dtype=np.int64)
        raw = self.ebsp_dataset[idx]
        if raw.dtype not in (np.float64, np.float32):
            raw = raw.astype(np.float64)
        src = torch.from_numpy(np.ascontiguousarray(raw))
        if out is None:
            return src
        dst = out[: src.numel()].view(src.shape)
        dst.copy_(src)
        return dst

    def to_device(self, host_raw: torch.Tensor) -> torch.Tensor:
        """(B, H0, W0) raw host batch -> (B, 1, h, w) fp32 device batch (DPdataset transform)."""
        if isinstance(self.transform, PatternTransform):
            return ingest_patterns(host_raw, self.image_size, self._dev())
        # a user transform: applied per pattern, as the reference's __getitem__ does
        return torch.stack([torch.as_tensor(self.transform(p.numpy().astype(np.float64)))
                            for p in host_raw]).to(self._dev())

    def batch(self, indices):
        """(patterns (B, 1, h, w) fp32 on device, angles (B, 3) float64) for `indices`."""
        idx = np.asarray(indices, dtype=np.int64)
        shape = (len(idx),) + tuple(self.ebsp_dataset.shape[1:])
        n = int(np.prod(shape))
        dt = torch.float32 if self.ebsp_dataset.dtype == np.float32 else torch.float64
        if self._pinned_free is not None:
            self._pinned_free.synchronize()   # the async copy of the previous batch read it
        if self._pinned is None or self._pinned.numel() < n or self._pinned.dtype != dt:
            self._pinned = torch.empty(n, dtype=dt).pin_memory()
        x = self.to_device(self.load_raw(idx, self._pinned))
        self._pinned_free = torch.cuda.Event()
        self._pinned_free.record()
        return x, self._angles[idx]

    def iter_batches(self, batch_size: int):
        for s in range(0, len(self), batch_size):
            yield self.batch(np.arange(s, min(s + batch_size, len(self))))


class DeviceBatchLoader:
    """The DataLoader of the drop-in DPDataModule: batches of (patterns on the device,
    angles (B, 3) float64 tensor) over a subset of a DPdataset, in order or shuffled per
    epoch.  A background thread reads batch i+1 from the memmap into the second of two
    pinned buffers while batch i is copied and transformed on the device; a buffer is
    refilled only after the device copy out of it has completed (HIP event).

    Order, matching what the reference's `DataLoader(..., shuffle=...)` yields
    (latice/data_module.py:215-261):
      * one process: `DataLoader(shuffle=True)` draws its base seed and then RandomSampler's
        seed from torch's default generator and permutes with a generator seeded by the
        latter; the same draws happen here, so torch.manual_seed(s) gives the same epoch
        order as the reference's loader.
      * torch.distributed initialised with W > 1 ranks (Lightning DDP, which would inject a
        DistributedSampler): each rank takes its DistributedSampler share -- the permutation
        of a generator seeded with seed + epoch (seed = PL_GLOBAL_SEED, as Lightning passes
        it, else 0), padded by wrapping to a multiple of W, then every W-th index from the
        rank's offset -- so the ranks see disjoint batches that cover the epoch.
        `set_epoch(e)` (reached through `.sampler`, where Lightning looks for it) moves to
        epoch e.
    Every torch DataLoader iterator draws a base seed from the default generator when it is
    created -- in order or shuffled, one process or W ranks -- except that a loader with
    persistent workers (the reference's val/test loaders when n_cpu > 0) creates its
    iterator once and draws it on the first iteration only; `persistent` says which.  Both
    draws (base seed, then RandomSampler's) happen when iter() is called, as DataLoader's
    worker iterator prefetches at creation, so later epochs and the other loaders see the
    reference's generator state."""

    def __init__(self, dataset: DPdataset, indices, batch_size: int, shuffle: bool = False,
                 drop_last: bool = False, rank: int | None = None, world: int | None = None,
                 seed: int | None = None, persistent: bool = False):
        self.dataset = dataset
        self.persistent = bool(persistent)
        self._iterated = False
        self.indices = np.asarray(indices, dtype=np.int64)
        self.batch_size = int(batch_size)
        self.shuffle = bool(shuffle)
        self.drop_last = bool(drop_last)
        if world is None:
            import torch.distributed as dist
            inited = dist.is_available() and dist.is_initialized()
            world = dist.get_world_size() if inited else 1
            rank = dist.get_rank() if inited else 0
        self.rank, self.world = int(rank or 0), int(world)
        if not 0 <= self.rank < self.world:
            raise ValueError(f"rank {self.rank} outside a world of {self.world}")
        import os
        self.seed = int(os.environ.get("PL_GLOBAL_SEED", 0)) if seed is None else int(seed)
        self.epoch = 0

    @property
    def sampler(self):
        return self

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def _num_local(self) -> int:
        n = len(self.indices)
        return n if self.world == 1 else math.ceil(n / self.world)

    def __len__(self) -> int:
        n = self._num_local()
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def _order(self):
        n = len(self.indices)
        if not (self.persistent and self._iterated):
            torch.empty((), dtype=torch.int64).random_()   # the iterator's base seed
        self._iterated = True
        if self.world > 1:
            # torch.utils.data.DistributedSampler (shuffle, drop_last=False)
            if self.shuffle:
                g = torch.Generator()
                g.manual_seed(self.seed + self.epoch)
                pos = torch.randperm(n, generator=g).numpy()
            else:
                pos = np.arange(n)
            total = self._num_local() * self.world
            if total > n:
                pos = np.concatenate([pos] * (total // n) + [pos[: total % n]])
            return self.indices[pos[self.rank:total:self.world]]
        if not self.shuffle:
            return self.indices
        # after the base seed, RandomSampler.__iter__ draws its own seed
        seed = int(torch.empty((), dtype=torch.int64).random_().item())
        g = torch.Generator()
        g.manual_seed(seed)
        return self.indices[torch.randperm(n, generator=g).numpy()]

    def __iter__(self):
        # the generator draws happen here, at iter(), not at the first next()
        return self._batches(self._order())

    def _batches(self, order):
        nb = len(self)
        if nb == 0:
            return
        ds = self.dataset
        shape = tuple(ds.ebsp_dataset.shape[1:])
        dt = torch.float32 if ds.ebsp_dataset.dtype == np.float32 else torch.float64
        per = int(np.prod(shape))
        bufs = [torch.empty(self.batch_size * per, dtype=dt).pin_memory() for _ in range(2)]
        done = [None, None]            # HIP event: device copy out of bufs[k] finished
        ready = [threading.Event(), threading.Event()]
        staged = [None, None]
        err = []

        def fill(i):
            k = i & 1
            try:
                if done[k] is not None:
                    done[k].synchronize()
                sel = np.sort(order[i * self.batch_size:(i + 1) * self.batch_size])
                staged[k] = (ds.load_raw(sel, bufs[k]), sel)
            except Exception as e:  # noqa: BLE001
                err.append(e)
            ready[k].set()

        th = threading.Thread(target=fill, args=(0,), daemon=True)
        th.start()
        for i in range(nb):
            k = i & 1
            ready[k].wait()
            th.join()
            if err:
                raise err[0]
            ready[k].clear()
            host, sel = staged[k]
            x = ds.to_device(host)
            ev = torch.cuda.Event()
            ev.record()
            done[k] = ev
            if i + 1 < nb:
                th = threading.Thread(target=fill, args=(i + 1,), daemon=True)
                th.start()
            yield x, torch.from_numpy(ds._angles[sel])


class DPDataModule(_DMBase):
    """data_module.py:136-261: same arguments, split and loaders; the loaders yield device
    batches (DeviceBatchLoader).  `n_cpu` starts no worker processes (one transform launch
    per batch replaces them); it only decides, as in the reference, whether the val/test
    loaders are persistent, which changes their generator draws."""

    def __init__(self, path, rot_angles_path, image_size=(128, 128), val_data_ratio: float = 0.1,
                 batch_size: int = 32, n_cpu: int = 4, seed: int = 42, transform=None,
                 device=None):
        super().__init__()
        self.path = path
        self.rot_angles_path = rot_angles_path
        self.image_size = tuple(image_size)
        self.val_data_ratio = val_data_ratio
        self.batch_size = batch_size
        self.n_cpu = n_cpu
        self.seed = seed
        self.transform = transform or create_default_transform(self.image_size)
        torch.manual_seed(seed)          # data_module.py:184-186
        np.random.seed(seed)
        self.dataset_full = DPdataset(self.path, self.rot_angles_path, self.image_size,
                                      self.transform, device=device)

    def setup(self, stage: str | None = None) -> None:
        """data_module.py:192-213 (random_split with a generator seeded by `seed`)."""
        if stage == "fit" or stage is None:
            all_size = len(self.dataset_full)
            val_size = int(all_size * self.val_data_ratio)
            train_size = all_size - val_size
            logger.info(f"Splitting dataset: {train_size} training, {val_size} validation samples")
            self.dataset_train, self.dataset_val = random_split(
                self.dataset_full, [train_size, val_size],
                generator=torch.Generator().manual_seed(self.seed))
        if stage == "test":
            self.dataset_test = self.dataset_full
            logger.info(f"Test dataset prepared with {len(self.dataset_test)} samples")

    def _loader(self, subset, shuffle):
        idx = subset.indices if hasattr(subset, "indices") else np.arange(len(subset))
        # val/test: persistent_workers=n_cpu > 0 (data_module.py:245,260)
        return DeviceBatchLoader(self.dataset_full, idx, self.batch_size, shuffle=shuffle,
                                 persistent=not shuffle and self.n_cpu > 0)

    def train_dataloader(self) -> DeviceBatchLoader:
        """data_module.py:215-233 (with no validation split, the whole set)."""
        if self.val_data_ratio > 0.0:
            return self._loader(self.dataset_train, shuffle=True)
        idx = np.concatenate([np.asarray(self.dataset_train.indices), np.asarray(self.dataset_val.indices)])
        return DeviceBatchLoader(self.dataset_full, idx, self.batch_size, shuffle=True)

    def val_dataloader(self) -> DeviceBatchLoader:
        return self._loader(self.dataset_val, shuffle=False)

    def test_dataloader(self) -> DeviceBatchLoader:
        return self._loader(self.dataset_test, shuffle=False)
