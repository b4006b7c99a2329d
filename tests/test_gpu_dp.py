"""Data-parallel equivalence of the benchmarked trainer on the GPU: two ranks (separate
processes, torch.distributed gloo, both on cuda:0) each run VAETrainer.forward_backward on
their half of a batch -- the loss kernel's gradient pre-scaled by 1/W, the two-bucket
all-reduce -- and must hold the single-process gradient of the whole batch.  Rank 1 starts
from different weights, so the init broadcast is checked too.
The RCCL ("nccl") path differs only in the backend string; it is exercised by the driver's
multi-GPU bench."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from latice.model import VariationalAutoEncoderRawData
from latice.seeding import seeded_eps, seeded_state_dict, synthetic_patterns
from latice.trainer import VAETrainer

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("prec", ["f16x3", "fp32"])
def test_two_rank_gradient_equals_single_process(cuda, tmp_path, prec):
    world, port = 2, _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), DP_OUT=str(tmp_path), DP_PREC=prec)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dp_trainer_worker.py")],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = [p.communicate(timeout=150)[0].decode() for p in procs]
    for p, out in zip(procs, outs):   # the tail of a failing worker's output, untruncated
        if p.returncode != 0:
            print(out[-6000:])
    assert all(p.returncode == 0 for p in procs), [o[-300:] for o in outs]
    from latice import engine as E
    with E.precision(prec):
        m = VariationalAutoEncoderRawData()
        m.load_state_dict({k: torch.from_numpy(v) for k, v in seeded_state_dict(0).items()})
        tr = VAETrainer(m.to(cuda), kl_lambda=5e-6)
        x = torch.from_numpy(synthetic_patterns(9, 4 * world)).to(cuda)
        eps = torch.from_numpy(seeded_eps(9, 4 * world)).to(cuda)
        loss, _, _ = tr.forward_backward(x, eps)
        g = tr.gflat.cpu().numpy().astype(np.float64)
    flat = [np.load(tmp_path / f"flat{r}.npy") for r in range(world)]
    assert np.array_equal(flat[0], flat[1])                       # broadcast at init
    assert np.array_equal(flat[0], tr.flat.cpu().numpy())
    for r in range(world):
        gr = np.load(tmp_path / f"gflat{r}.npy").astype(np.float64)
        err = np.abs(gr - g).max() / np.abs(g).max()
        print(f"\nrank {r} all-reduced gradient vs single process 2B: {err:.2e}")
        assert err < 1e-5
    losses = [float(np.load(tmp_path / f"loss{r}.npy")[0]) for r in range(world)]
    assert abs(np.mean(losses) - float(loss)) < 1e-6 * abs(float(loss))
