"""Poison mode (EBSDVAE_POISON / engine.set_poison): every buffer the engine hands to a
kernel -- activations, gradients, InstanceNorm statistics, weight-gradient slice partials,
fused-reduce sums, split-K scratch -- is NaN-filled when it is allocated, and the trainer
NaN-fills its flat gradient buffer before each step.  A kernel that leaves any element of
its output unwritten, or a consumer (on either stream) that reads a buffer before its
producer wrote it, then turns a result into NaN instead of into a small, in-tolerance error
from whatever the caching allocator's block last held.

This is the check VERDICT r05 asked for after one fp32 run of
test_trainer_forward_backward_vs_pinned_oracle[vae128_b8_c1-fp32] returned decoder.13.0's
weight gradient 200x further from the oracle than every other run.
Each case runs once; the pinned gates of tests/pinned.py apply unchanged.
"""
import pytest
import torch

from pinned import check_grads, fixture
from latice import engine as E
from latice.model import VariationalAutoEncoderRawData
from latice.trainer import VAETrainer

pytestmark = pytest.mark.gpu


@pytest.fixture
def poison():
    E.set_poison(True)
    try:
        yield
    finally:
        E.set_poison(False)


def _model(name, device):
    f, sd = fixture(name)
    B, S, L, ws, xs = (int(v) for v in f["meta"])
    m = VariationalAutoEncoderRawData(32, L, S)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return f, m.to(device)


def _finite(tr):
    bad = [n for n, g in tr.G.items() if not torch.isfinite(g).all()]
    assert not bad, f"gradients with unwritten (NaN) entries: {bad}"


@pytest.mark.parametrize("prec", ["f16x3", "bf16x6", "fp32"])
@pytest.mark.parametrize("name", ["vae128_b4", "vae128_b8_c1", "vae256_b2_l64"])
def test_trainer_step_under_poison(cuda, poison, name, prec):
    f, m = _model(name, cuda)
    x = torch.from_numpy(f["x"]).to(cuda)
    eps = torch.from_numpy(f["eps"]).to(cuda)
    with E.precision(prec):
        tr = VAETrainer(m, kl_lambda=float(f["kl_lambda"]))
        with E.record_state() as rec:
            loss, kl, rec_loss = tr.forward_backward(x, eps)
        torch.cuda.synchronize()
    for k, v in (("loss", loss), ("kl_loss", kl), ("recon_loss", rec_loss)):
        assert abs(float(v) - float(f[k])) <= 1e-5 * abs(float(f[k])) + 1e-12, k
    _finite(tr)
    check_grads(name, m.plan, rec, tr.G, label=f"poison {prec}", prec=prec)


@pytest.mark.parametrize("prec", ["f16x3", "fp32"])
def test_full_size_step_under_poison(cuda, poison, prec):
    """B = 256 (the bench shape: whole-image persistent blocks, in-kernel finalize, every
    slice count of the production launches) -- two consecutive steps, so the second one's
    buffers come back from the caching allocator (NaN-filled again) instead of fresh."""
    from latice.seeding import seeded_eps, seeded_state_dict, synthetic_patterns
    m = VariationalAutoEncoderRawData().to(cuda)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in seeded_state_dict(0).items()})
    x = torch.from_numpy(synthetic_patterns(3, 256)).to(cuda)
    eps = torch.from_numpy(seeded_eps(3, 256)).to(cuda)
    with E.precision(prec):
        tr = VAETrainer(m, kl_lambda=5e-6)
        g = []
        for _ in range(2):
            loss, _, _ = tr.forward_backward(x, eps)
            torch.cuda.synchronize()
            assert torch.isfinite(loss)
            _finite(tr)
            g.append(tr.gflat.clone())
    assert torch.equal(g[0], g[1]), "the same step gave different gradients"


def test_autograd_drop_in_and_encoder_under_poison(cuda, poison):
    """The nn.Module drop-in (autograd path, latice.functional) and the encoder-only
    inference path (c4) under poison: every output and parameter gradient is written."""
    f, m = _model("vae128_b4", cuda)
    x = torch.from_numpy(f["x"]).to(cuda)
    z, x_hat, mu, std = m(x)
    (x_hat.float().mean() + z.square().mean() + mu.square().mean() + std.mean()).backward()
    torch.cuda.synchronize()
    for t in (z, x_hat, mu, std):
        assert torch.isfinite(t).all()
    bad = [n for n, p in m.named_parameters() if p.grad is None or not torch.isfinite(p.grad).all()]
    assert not bad, bad
    m.eval()
    with torch.no_grad():
        mu = m(x.repeat(256, 1, 1, 1).contiguous())[2]
    torch.cuda.synchronize()
    assert torch.isfinite(mu).all()
