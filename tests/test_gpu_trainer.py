"""Parity of the BENCHMARKED path: `VAETrainer.forward_backward` (what bench.py times) --
the batched PackSet weight packs, the split-fp16 forward, the scaled split-fp16 input
gradient, the f16 weight gradient, the flat gradient buffer and the loss kernel's 1/W
scale -- against the reference's golden fixtures and the pinned float64 oracle
(tests/pinned.py: every non-bias weight gradient <= 1e-3 decision-pinned and <= 1e-4
state-pinned, zero-grad bias residues <= ZERO_BIAS_K[arithmetic] x 2^-24 sum|gy|).
"""
import numpy as np
import pytest
import torch

from pinned import check_grads, fixture, host
from latice import engine as E
from latice.model import VariationalAutoEncoderRawData
from latice.trainer import VAETrainer
from oracle import vae_oracle as O

pytestmark = pytest.mark.gpu

FIXTURES = ["vae128_b4", "vae128_b8_c1", "vae128_b2_edge", "vae256_b2_l64"]


def build(name, device):
    f, sd = fixture(name)
    B, S, L, ws, xs = (int(v) for v in f["meta"])
    m = VariationalAutoEncoderRawData(32, L, S)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return f, m.to(device)


@pytest.mark.parametrize("prec", ["f16x3", "bf16x6", "fp32"])
@pytest.mark.parametrize("name", FIXTURES)
def test_trainer_forward_backward_vs_pinned_oracle(cuda, name, prec):
    f, m = build(name, cuda)
    x = torch.from_numpy(f["x"]).to(cuda)
    eps = torch.from_numpy(f["eps"]).to(cuda)
    with E.precision(prec):
        tr = VAETrainer(m, kl_lambda=float(f["kl_lambda"]))
        if prec == "f16x3":   # the benchmarked arithmetic: f16 packs for the input gradients
            f16 = [L.name for L in m.plan.enc[1:] + m.plan.dec[:-1]
                   if tr.packset.packs[L.name][1].pieces == E.PIECES_F16]
            assert f16, "no split-fp16 input-gradient pack under f16x3"
        with E.record_state() as rec:
            loss, kl, rec_loss = tr.forward_backward(x, eps)
        torch.cuda.synchronize()
    for k, v in (("loss", loss), ("kl_loss", kl), ("recon_loss", rec_loss)):
        ref = float(f[k])
        assert abs(float(v) - ref) <= 1e-5 * abs(ref) + 1e-12, k
    check_grads(name, m.plan, rec, tr.G, label=f"trainer {prec}", prec=prec)


def test_trainer_step_is_adam_on_the_checked_gradient(cuda):
    """One trainer.step == forward_backward + torch.optim.Adam(lr 1e-4) on the same flat
    gradient (the fused Adam of the benchmarked step)."""
    f, m = build("vae128_b4", cuda)
    x = torch.from_numpy(f["x"]).to(cuda)
    eps = torch.from_numpy(f["eps"]).to(cuda)
    tr = VAETrainer(m, kl_lambda=float(f["kl_lambda"]), lr=1e-4)
    p0 = tr.flat.clone()
    tr.forward_backward(x, eps)
    g = tr.gflat.clone()
    tr.optimizer_step()
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=1e-4, foreach=False)
    ref.grad = g
    opt.step()
    torch.cuda.synchronize()
    assert torch.allclose(tr.flat, ref.detach(), rtol=1e-6, atol=1e-9)


def test_trainer_full_size_gradient_batch_independence(cuda):
    """B=256 (the bench config): with the per-sample loss scale 1/B, the gradient of the
    full batch equals the mean of the gradients of its two halves (the same property the
    data-parallel all-reduce relies on): a size-independent check of the full-size backward."""
    from latice.seeding import seeded_eps, seeded_state_dict, synthetic_patterns
    sd = {k: torch.from_numpy(v) for k, v in seeded_state_dict(0).items()}
    m = VariationalAutoEncoderRawData().to(cuda)
    m.load_state_dict(sd)
    tr = VAETrainer(m, kl_lambda=5e-6)
    x = torch.from_numpy(synthetic_patterns(3, 256)).to(cuda)
    eps = torch.from_numpy(seeded_eps(3, 256)).to(cuda)
    tr.forward_backward(x, eps)
    g_full = tr.gflat.clone()
    halves = []
    for h in range(2):
        sl = slice(128 * h, 128 * (h + 1))
        tr.forward_backward(x[sl].contiguous(), eps[sl].contiguous())
        halves.append(tr.gflat.clone())
    torch.cuda.synchronize()
    g_mean = 0.5 * (halves[0] + halves[1])
    err = float((g_full - g_mean).abs().max() / g_mean.abs().max())
    print(f"\nfull-batch gradient vs mean of halves: {err:.2e}")
    assert np.isfinite(err) and err < 1e-4


@pytest.mark.parametrize("prec", ["f16x3", "fp32"])
def test_trainer_network_end_fusion_matches_separate_kernels(cuda, prec, monkeypatch):
    """The fused network end (ebsdvae_net_end) and the separate final conv / loss / reduce
    kernels give the same step: loss scalars and every gradient within fp32 reordering."""
    from latice.seeding import seeded_eps, seeded_state_dict, synthetic_patterns
    sd = {k: torch.from_numpy(v) for k, v in seeded_state_dict(0).items()}
    x = torch.from_numpy(synthetic_patterns(4, 16)).to(cuda)
    eps = torch.from_numpy(seeded_eps(4, 16)).to(cuda)
    out = {}
    with E.precision(prec):
        for fused in (True, False):
            monkeypatch.setattr(E, "_NET_END", fused)
            m = VariationalAutoEncoderRawData().to(cuda)
            m.load_state_dict(sd)
            tr = VAETrainer(m, kl_lambda=5e-6)
            assert E.net_end_ok(m.plan) == fused   # 128x128: the fused kernel's shape
            loss, kl, rec = tr.forward_backward(x, eps)
            torch.cuda.synchronize()
            out[fused] = ([float(loss), float(kl), float(rec)], tr.gflat.clone(), dict(tr.G))
    (l1, g1, G1), (l0, g0, G0) = out[True], out[False]
    for a, b in zip(l1, l0):
        assert abs(a - b) <= 1e-6 * abs(b) + 1e-12
    worst = max(O.rel_err(host(G1[n]), host(G0[n])) for n in G1 if n.endswith("weight"))
    print(f"\n[{prec}] fused vs separate network end: worst weight-grad rel err {worst:.2e}")
    assert worst < 1e-4
