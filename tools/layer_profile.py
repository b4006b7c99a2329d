"""Per-layer timing of the conv kernels inside one training step (HIP events around each
launch, engine.probe), as TFLOP/s against the fp32 MFMA peak.

    python tools/layer_profile.py [--batch 256] [--steps 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ebsd-vae_amd")]

import torch  # noqa: E402

from latice import engine as E  # noqa: E402
from latice.model import VariationalAutoEncoderRawData  # noqa: E402
from latice.seeding import seeded_state_dict, synthetic_patterns  # noqa: E402
from latice.trainer import VAETrainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--image-size", type=int, default=128)
    ap.add_argument("--latent-dim", type=int, default=16)
    ap.add_argument("--serial", action="store_true",
                    help="weight gradients on the main stream (each launch timed alone)")
    a = ap.parse_args()
    m = VariationalAutoEncoderRawData(32, a.latent_dim, a.image_size)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in
                       seeded_state_dict(0, 32, a.latent_dim, a.image_size).items()})
    m = m.cuda()
    tr = VAETrainer(m)
    x = torch.from_numpy(synthetic_patterns(0, a.batch, a.image_size)).cuda()
    for _ in range(2):
        tr.step(x)
    import contextlib
    with E.probe() as pr, (E.serial_streams() if a.serial else contextlib.nullcontext()):
        for _ in range(a.steps):
            tr.step(x)
    rows = sorted(pr.per_tag().items(), key=lambda kv: -kv[1][2])
    tot = sum(v[2] for _, v in rows) / a.steps
    print(f"{'tag':58s} {'ms/step':>8s} {'TF/s':>7s}")
    for tag, (n, fl, ms) in rows:
        print(f"{tag:58s} {ms / a.steps:8.3f} {fl / (ms / 1e3) / 1e12:7.1f}")
    print(f"{'total conv kernels':58s} {tot:8.3f}")


if __name__ == "__main__":
    main()
