"""The CPU-baseline port (oracle/torch_port.py) reproduces the reference's golden
vectors, so bench.py's cpu_baseline times the same computation."""
import os

import numpy as np
import torch

from conftest import GOLDEN
from latice.seeding import seeded_state_dict
from oracle import torch_port as TP
from oracle import vae_oracle as O


def test_torch_port_matches_golden():
    f = O.load_fixture(os.path.join(GOLDEN, "vae128_b4.npz"))
    B, S, L, ws, xs = (int(v) for v in f["meta"])
    sd = seeded_state_dict(ws, 32, L, S)
    p = {k: torch.from_numpy(v).double().requires_grad_(True) for k, v in sd.items()}
    x = torch.from_numpy(f["x"]).double()
    z, xh, mu, std = TP.forward(p, x, torch.from_numpy(f["eps"]).double())
    assert O.rel_err(mu.detach().numpy(), f["mu"]) < 1e-10
    assert O.rel_err(xh.detach().numpy(), f["x_hat"]) < 1e-6
    out = TP.loss(z, xh, mu, std, x, float(f["kl_lambda"]))
    assert abs(float(out["loss"]) - float(f["loss"])) < 1e-10
    out["loss"].backward()
    g = p["encoder.4.0.weight"].grad.numpy().ravel()
    assert O.rel_err(g[f["grad_idx/encoder.4.0.weight"]], f["grad_sub/encoder.4.0.weight"]) < 1e-6


def test_cpu_step_runs():
    sd = seeded_state_dict(0)
    st = TP.CPUStep(sd)
    x = torch.rand(2, 1, 128, 128)
    l0 = st.step(x, torch.zeros(2, 16))
    l1 = st.step(x, torch.zeros(2, 16))
    assert np.isfinite(l0) and np.isfinite(l1)


def test_cpu_encoder_matches_reference_mu():
    """CPUStep.encode (the c4 cpu_baseline leg) == the reference's mu on the golden fixture."""
    f = O.load_fixture(os.path.join(GOLDEN, "vae128_b4.npz"))
    B, S, L, ws, xs = (int(v) for v in f["meta"])
    st = TP.CPUStep(seeded_state_dict(ws, 32, L, S))
    mu = st.encode(torch.from_numpy(f["x"]))
    assert O.rel_err(mu.numpy(), f["mu"]) < 1e-5
