"""Data-parallel path on CPU (torch.distributed gloo, world size 2).

* GradReducer: the two-bucket async SUM all-reduce of the flat gradient buffer used by
  latice.trainer.VAETrainer (RCCL on the GPU box).
* DP equivalence: each rank back-propagates its shard with the loss gradient pre-scaled
  by 1/W (what VAETrainer passes to the loss kernel); the SUM all-reduce then equals the
  single-process gradient of the global batch.  Checked with the float64 oracle.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import sys
    for p in (ROOT, os.path.join(ROOT, "ebsd-vae_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _reducer_worker(rank, world, port, q):
    _init(rank, world, port)
    from latice.trainer import GradReducer, shard_batch
    g = torch.arange(11, dtype=torch.float32) * (rank + 1)
    r = GradReducer(g, split=4)
    r.start(0)
    r.start(1)
    r.finish()
    # three buckets (the trainer's decoder+heads / deep encoder / shallow encoder split),
    # started out of order like the hooks can; an empty bucket is skipped
    g3 = torch.arange(13, dtype=torch.float32) * (rank + 1)
    r3 = GradReducer(g3, split=[3, 9, 9])
    r3.start(1)
    r3.start(0)
    r3.start(2)
    r3.start(3)
    r3.finish()
    x = torch.arange(8).reshape(8, 1)
    q.put((rank, g.numpy().copy(), shard_batch(x, rank, world).numpy().ravel().tolist(),
           g3.numpy().copy()))
    dist.destroy_process_group()


def _dp_worker(rank, world, port, q):
    _init(rank, world, port)
    from latice.seeding import seeded_eps, seeded_state_dict, synthetic_patterns
    from latice.trainer import GradReducer
    from oracle import vae_oracle as O
    sd = seeded_state_dict(0)
    x = synthetic_patterns(5, 2 * world)
    eps = seeded_eps(5, 2 * world)
    lo, hi = 2 * rank, 2 * rank + 2
    _, cache = O.forward(sd, x[lo:hi], eps[lo:hi])
    g = O.backward(cache, x[lo:hi], 0.1, g_loss=1.0 / world)
    names = list(sd)
    flat = torch.from_numpy(np.concatenate([g[n].ravel() for n in names]))
    r = GradReducer(flat, split=flat.numel() // 3)
    r.start(0)
    r.start(1)
    r.finish()
    q.put((rank, flat.numpy()))
    dist.destroy_process_group()


def _run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda t: t[0])


def test_grad_reducer_two_buckets_sum():
    out = _run(_reducer_worker)
    expect = np.arange(11, dtype=np.float32) * 3
    for rank, g, shard, g3 in out:
        assert np.array_equal(g, expect)
        assert shard == list(range(4 * rank, 4 * rank + 4))
        assert np.array_equal(g3, np.arange(13, dtype=np.float32) * 3)


def test_grad_reducer_rejects_bad_boundaries():
    from latice.trainer import GradReducer
    with pytest.raises(ValueError, match="increase"):
        GradReducer(torch.zeros(10), split=[6, 3])
    with pytest.raises(ValueError, match="increase"):
        GradReducer(torch.zeros(10), split=[12])


@pytest.mark.timeout(600)
def test_dp_sharded_gradient_equals_global_gradient():
    out = _run(_dp_worker)
    import sys
    for p in (ROOT, os.path.join(ROOT, "ebsd-vae_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from latice.seeding import seeded_eps, seeded_state_dict, synthetic_patterns
    from oracle import vae_oracle as O
    sd = seeded_state_dict(0)
    x = synthetic_patterns(5, 4)
    eps = seeded_eps(5, 4)
    _, cache = O.forward(sd, x, eps)
    g = O.backward(cache, x, 0.1)
    ref = np.concatenate([g[n].ravel() for n in sd])
    for _, flat in out:
        assert np.array_equal(out[0][1], flat)          # every rank holds the same gradient
        assert O.rel_err(flat, ref) < 1e-10
