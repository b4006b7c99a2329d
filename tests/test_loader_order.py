"""Batch order of the drop-in DPDataModule loaders (latice.data_module.DeviceBatchLoader)
against what the reference's torch DataLoader would yield (latice/data_module.py:215-261):
one process = DataLoader(shuffle=...) under the same torch.manual_seed; W ranks = the
DistributedSampler share Lightning DDP injects.  CPU only: the order is host logic."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from torch.utils.data import DataLoader, DistributedSampler, TensorDataset

from latice.data_module import DeviceBatchLoader


def _ref_order(n, bs, shuffle, seed):
    torch.manual_seed(seed)
    dl = DataLoader(TensorDataset(torch.arange(n)), batch_size=bs, shuffle=shuffle)
    return [b[0].tolist() for b in dl]


def _mine(loader):
    o = loader._order()
    return [o[i:i + loader.batch_size].tolist() for i in range(0, len(o), loader.batch_size)]


@pytest.mark.parametrize("shuffle", [True, False])
def test_single_process_order_matches_dataloader(shuffle):
    n, bs = 103, 16
    ref = _ref_order(n, bs, shuffle, seed=42)
    torch.manual_seed(42)
    ld = DeviceBatchLoader(None, np.arange(n), bs, shuffle=shuffle, rank=0, world=1)
    got = _mine(ld)
    assert got == ref and len(ld) == len(ref)
    # consecutive epochs keep following the reference's generator
    torch.manual_seed(7)
    dl = DataLoader(TensorDataset(torch.arange(n)), batch_size=bs, shuffle=shuffle)
    ref2 = [[b[0].tolist() for b in dl] for _ in range(2)]
    torch.manual_seed(7)
    assert [_mine(ld) for _ in range(2)] == ref2


@pytest.mark.parametrize("shuffle", [True, False])
@pytest.mark.parametrize("n", [100, 101, 3])
def test_rank_shares_match_distributed_sampler(shuffle, n):
    world, bs = 4, 8
    idx = np.arange(1000, 1000 + n)          # a subset's indices, as random_split gives
    for epoch in (0, 3):
        seen = []
        for r in range(world):
            ds = DistributedSampler(TensorDataset(torch.arange(n)), num_replicas=world, rank=r,
                                    shuffle=shuffle, seed=0)
            ds.set_epoch(epoch)
            ref = idx[np.asarray(list(ds))]
            ld = DeviceBatchLoader(None, idx, bs, shuffle=shuffle, rank=r, world=world, seed=0)
            ld.sampler.set_epoch(epoch)      # where Lightning calls it
            assert np.array_equal(ld._order(), ref)
            assert len(ld) == -(-len(ref) // bs)
            seen.append(ld._order())
        allx = np.concatenate(seen)
        assert set(allx.tolist()) == set(idx.tolist())     # the epoch is covered
        if n % world == 0:
            assert len(allx) == n                          # and, unpadded, disjoint


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ld = DeviceBatchLoader(None, np.arange(64), 8, shuffle=True)   # rank/world from the group
        out[rank] = (ld.rank, ld.world, ld._order().tolist())
    finally:
        dist.destroy_process_group()


def test_two_rank_group_gives_disjoint_batches():
    world = 2
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(world, _port(), out), nprocs=world, join=True)
        res = dict(out)
    assert [res[r][:2] for r in range(world)] == [(0, 2), (1, 2)]
    a, b = res[0][2], res[1][2]
    assert not set(a) & set(b) and sorted(a + b) == list(range(64))


@pytest.mark.parametrize("n_cpu", [0, 1])
def test_val_then_train_follow_reference_generator(n_cpu):
    """Lightning's fit: a sanity-check pass over the val loader, then per epoch the train
    loader and the val loader.  Every DataLoader iterator draws a base seed, the persistent
    val loader (n_cpu > 0) only on its first iteration (data_module.py:225-246)."""
    n_tr, n_va, bs, seed = 37, 11, 8, 3
    torch.manual_seed(seed)
    tr = DataLoader(TensorDataset(torch.arange(n_tr)), batch_size=bs, shuffle=True, num_workers=n_cpu)
    va = DataLoader(TensorDataset(torch.arange(n_va)), batch_size=bs, shuffle=False,
                    num_workers=n_cpu, persistent_workers=n_cpu > 0)
    ref = [[b[0].tolist() for b in va]]
    for _ in range(2):
        ref.append([b[0].tolist() for b in tr])
        ref.append([b[0].tolist() for b in va])
    ref_next = torch.rand(3)
    del tr, va

    torch.manual_seed(seed)
    mtr = DeviceBatchLoader(None, np.arange(n_tr), bs, shuffle=True, rank=0, world=1)
    mva = DeviceBatchLoader(None, np.arange(n_va), bs, shuffle=False, rank=0, world=1,
                            persistent=n_cpu > 0)
    got = [_mine(mva)]
    for _ in range(2):
        got.append(_mine(mtr))
        got.append(_mine(mva))
    assert got == ref
    assert torch.equal(torch.rand(3), ref_next)     # the generator ends in the same state
