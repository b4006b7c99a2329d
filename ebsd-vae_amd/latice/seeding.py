"""Deterministic, version-stable parameter initialisation from a seed.

PyTorch's default init (kaiming-uniform a=sqrt(5) for weights, U(+-1/sqrt(fan_in))
for biases) is what the reference model actually ends up with: its
``weights_init`` hook (`latice/model.py:68-80`) is applied at `latice/model.py:16`,
before any submodule exists, so it never touches a layer.  Here the same bounds
are drawn from numpy's PCG64 (stable across numpy/torch versions), so the golden
fixtures, the oracle, the tests and the benchmark all regenerate bit-identical
weights from an integer seed without shipping a weight file.

Parameter order and shapes follow the 46-key state_dict of
`VariationalAutoEncoderRawData` (`latice/model.py:109-150`).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np

# (key prefix, kind, cin, cout) with kind in {"conv", "convT"}; spatial scale factor
# relative to the input is only needed by the model, not by the init.
_ENC_IDX = (0, 1, 3, 4, 6, 7, 9, 10, 12, 13)
_DEC_IDX = (1, 2, 4, 5, 7, 8, 10, 11, 13)


def layer_table(inplanes: int = 32, latent_dim: int = 16, image_size: int = 128):
    """Return the ordered parameter table [(name, shape, fan_in)].

    Mirrors `latice/model.py:109-150` (encoder / mu / logvar / linear2 / decoder).
    ``image_size`` only changes the flattened feature width (the reference
    hard-codes 128x128 -> 4x4, `latice/model.py:127-131`; 256x256 gives 8x8).
    """
    p = inplanes
    enc = [(1, p), (p, p), (p, 2 * p), (2 * p, 2 * p), (2 * p, 4 * p), (4 * p, 4 * p),
           (4 * p, 4 * p), (4 * p, 4 * p), (4 * p, 4 * p), (4 * p, 4 * p)]
    dec = [(4 * p, 4 * p), (4 * p, 4 * p), (4 * p, 4 * p), (4 * p, 4 * p), (4 * p, 4 * p),
           (4 * p, 2 * p), (2 * p, 2 * p), (2 * p, p), (p, p)]
    side = image_size // 32
    flat = 4 * p * side * side
    rows = []
    for idx, (ci, co) in zip(_ENC_IDX, enc):
        rows.append((f"encoder.{idx}.0.weight", (co, ci, 3, 3), ci * 9))
        rows.append((f"encoder.{idx}.0.bias", (co,), ci * 9))
    rows.append(("mu.0.weight", (latent_dim, flat), flat))
    rows.append(("mu.0.bias", (latent_dim,), flat))
    rows.append(("logvar.0.weight", (latent_dim, flat), flat))
    rows.append(("logvar.0.bias", (latent_dim,), flat))
    rows.append(("linear2.0.weight", (flat, latent_dim), latent_dim))
    rows.append(("linear2.0.bias", (flat,), latent_dim))
    for idx, (ci, co) in zip(_DEC_IDX, dec):
        # ConvTranspose2d weight is (Cin, Cout, 3, 3); torch's fan_in uses dim 1.
        rows.append((f"decoder.{idx}.0.weight", (ci, co, 3, 3), co * 9))
        rows.append((f"decoder.{idx}.0.bias", (co,), co * 9))
    rows.append(("decoder.14.weight", (1, p, 3, 3), p * 9))
    rows.append(("decoder.14.bias", (1,), p * 9))
    return rows


def seeded_state_dict(seed: int, inplanes: int = 32, latent_dim: int = 16,
                      image_size: int = 128) -> "OrderedDict[str, np.ndarray]":
    """Draw every parameter U(-1/sqrt(fan_in), +1/sqrt(fan_in)) in state_dict order."""
    rng = np.random.default_rng(seed)
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for name, shape, fan_in in layer_table(inplanes, latent_dim, image_size):
        bound = 1.0 / math.sqrt(fan_in)
        out[name] = rng.uniform(-bound, bound, size=shape).astype(np.float32)
    return out


def synthetic_patterns(seed: int, batch: int, image_size: int = 128) -> np.ndarray:
    """Uniform [0,1) patterns quantised to k/255, shape (B,1,S,S) float32.

    Mimics the DPdataset pipeline output (`latice/data_module.py:17-33,122-133`:
    ToPILImage -> uint8 -> ToTensor gives multiples of 1/255).
    """
    rng = np.random.default_rng(seed)
    u = rng.random((batch, 1, image_size, image_size))
    return (np.floor(u * 255.0) / 255.0).astype(np.float32)


def seeded_eps(seed: int, batch: int, latent_dim: int = 16) -> np.ndarray:
    """Standard-normal reparameterisation noise (B, latent) float32 for parity runs."""
    rng = np.random.default_rng(seed + 7919)
    return rng.standard_normal((batch, latent_dim)).astype(np.float32)
