"""Record the reference's own fp32 rounding noise on the analytically-zero conv biases at the
benchmarked batch (this container only; imports the reference like make_golden.py).

Every conv that feeds an affine-free InstanceNorm (latice/model.py:109-148) has a bias whose
gradient is exactly zero: IN subtracts the per-(image, channel) mean, so d loss / d bias_c =
sum over (b, h, w) of gy[b, c, h, w] = 0.  An fp32 backward returns the rounding residue of
that sum.  Its size scales with the magnitude of what is summed, so the parity gate for these
biases (tests/pinned.py) is relative to  A_c = sum over (b, h, w) of |gy[b, c, h, w]|  (the
float64 run's), not an absolute number.  This script runs the reference at B=256 (config c2,
128x128, latent 16, seeded weights and patterns of latice/seeding.py) in float64 and float32
and stores, per zero-gradient bias: A_c (float64), |db_c| of the float32 run, and |db_c| of
the float64 run -- the reference's own noise floor in units of 2^-24 * A_c.

    python tests/golden/make_bias_noise.py [--batch 256]   ->  tests/golden/bias_noise_b256.npz
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import _VariantVAE, _import_reference, _load_seeding  # noqa: E402


def zero_bias_convs(model):
    """(state_dict prefix, Conv2d / ConvTranspose2d) of every conv followed by InstanceNorm."""
    import torch.nn as nn
    out = []
    for part in ("encoder", "decoder"):
        seq = getattr(model, part)
        for i, blk in enumerate(seq):
            if isinstance(blk, nn.Sequential) and any(isinstance(m, nn.InstanceNorm2d) for m in blk):
                out.append((f"{part}.{i}.0", blk[0]))
    return out


def run(ref_model, ref_lm, seeding, batch, dtype):
    import torch
    import torch.distributions.normal as tdn
    sd = seeding.seeded_state_dict(0, 32, 16, 128)
    x = seeding.synthetic_patterns(3, batch, 128)
    eps = seeding.seeded_eps(3, batch, 16)
    model = _VariantVAE.build(ref_model, 32, 16, 128)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model = model.to(dtype)
    absum = {}
    hooks = []
    for name, conv in zero_bias_convs(model):
        def fwd_hook(mod, inp, out, name=name):
            out.register_hook(lambda g, name=name: absum.__setitem__(
                name, g.detach().abs().sum(dim=(0, 2, 3)).double().numpy()))
        hooks.append(conv.register_forward_hook(fwd_hook))
    et = torch.from_numpy(eps).to(dtype)
    orig = tdn._standard_normal
    tdn._standard_normal = lambda shape, dtype, device: et.clone()
    try:
        z, x_hat, mu, std = model(torch.from_numpy(x).to(dtype))
    finally:
        tdn._standard_normal = orig
    loss = ref_lm.VAELoss(kl_lambda=5e-6).compute_loss(z, x_hat, mu, std, torch.from_numpy(x).to(dtype))
    loss["loss"].backward()
    for h in hooks:
        h.remove()
    db = {name: conv.bias.grad.detach().double().numpy().copy() for name, conv in zero_bias_convs(model)}
    return absum, db


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    import torch
    torch.set_num_threads(8)
    seeding = _load_seeding()
    ref_model, ref_lm = _import_reference(a.ref)
    a64, d64 = run(ref_model, ref_lm, seeding, a.batch, torch.float64)
    _, d32 = run(ref_model, ref_lm, seeding, a.batch, torch.float32)
    out = {"batch": np.array(a.batch), "names": np.array(sorted(a64))}
    u = 2.0 ** -24
    for n in sorted(a64):
        out["absum/" + n] = a64[n]
        out["db64/" + n] = d64[n]
        out["db32/" + n] = d32[n]
        r = np.abs(d32[n]) / (u * a64[n])
        print(f"{n:14s} A max {a64[n].max():.3e}  |db32| max {np.abs(d32[n]).max():.2e}  "
              f"|db32|/(2^-24 A) max {r.max():.3f}  |db64| max {np.abs(d64[n]).max():.1e}")
    path = os.path.join(HERE, f"bias_noise_b{a.batch}.npz")
    np.savez_compressed(path, **out)
    print("wrote", path)


if __name__ == "__main__":
    main()
