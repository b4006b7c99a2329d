"""Dump the flat gradient of one benchmarked training step (c2 shapes, fixed seeds) to an .npy
file: run it under two libraries (EBSDVAE_LIB) and compare the files for a bitwise A/B.
    python tools/gflat_dump.py OUT.npy"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ebsd-vae_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from latice.model import VariationalAutoEncoderRawData  # noqa: E402
from latice.seeding import seeded_eps, seeded_state_dict, synthetic_patterns  # noqa: E402
from latice.trainer import VAETrainer  # noqa: E402

dev = torch.device("cuda")
m = VariationalAutoEncoderRawData(32, 16, 128)
m.load_state_dict({k: torch.from_numpy(v) for k, v in seeded_state_dict(0, 32, 16, 128).items()})
m = m.to(dev)
x = torch.from_numpy(synthetic_patterns(3, 256)).to(dev)
eps = torch.from_numpy(seeded_eps(3, 256)).to(dev)
tr = VAETrainer(m, kl_lambda=5e-6)
loss = tr.forward_backward(x, eps)
torch.cuda.synchronize()
np.save(sys.argv[1], tr.gflat.cpu().numpy())
print("loss", [float(v) for v in loss])
