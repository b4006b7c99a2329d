"""The second conv block's forward with the first block recomputed from x
(ebsdvae_conv3x3_fwd_split_first, engine.conv_forward_first): every staged value is the first
conv's own fma chain (ebsdvae_conv_first_fwd) followed by the same normalisation, so the
block's outputs must be BITWISE those of the two-launch form that writes y0 and reads it back
(EBSDVAE_FIRST_FUSE=0).  The default uses it in inference only ("eval": the first conv then
writes no y0 at all); "1" also in training.  Checked at the bench shapes -- c2 (128^2, B = 256: whole-image
persistent blocks, in-kernel finalize), c4's encoder-only inference (no y0 at all) and c5
(256^2, four staged items per thread) -- and on a ragged batch (B = 5: the standalone finalize).
"""
import pytest
import torch

from latice import engine as E
from latice.model import VariationalAutoEncoderRawData
from latice.seeding import seeded_eps, seeded_state_dict, synthetic_patterns
from latice.trainer import VAETrainer

pytestmark = pytest.mark.gpu


def _model(cuda, S, L):
    m = VariationalAutoEncoderRawData(32, L, S)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in seeded_state_dict(0, 32, L, S).items()})
    return m.to(cuda)


def _encode(m, x, train, fuse, monkeypatch):
    monkeypatch.setattr(E, "_FIRST_FUSE", "1" if fuse else "0")
    params = dict(m.named_parameters())
    with E.record_launches() as launches:
        out, saved = E.encoder_forward(m.plan, x, params, train=train)
    torch.cuda.synchronize()
    assert ("ebsdvae_conv3x3_fwd_split_first" in launches) == fuse
    return out, saved, launches


@pytest.mark.parametrize("S,L,B", [(128, 16, 256), (128, 16, 5), (256, 64, 8)],
                         ids=["c2-B256", "ragged-B5", "c5-256px"])
@pytest.mark.parametrize("train", [True, False], ids=["train", "eval"])
def test_first_fuse_is_bitwise(cuda, monkeypatch, S, L, B, train):
    m = _model(cuda, S, L)
    assert E.first_fuse_ok(m.plan, E.pack_weight(m.encoder[1][0].weight, m.plan.enc[1], dgrad=False))
    x = torch.from_numpy(synthetic_patterns(1, B, S)).to(cuda)
    with torch.no_grad():
        o1, s1, _ = _encode(m, x, train, True, monkeypatch)
        o0, s0, _ = _encode(m, x, train, False, monkeypatch)
    assert torch.equal(o1, o0), "encoder output differs"
    assert set(s1) == set(s0)
    for k in s0:
        a, b = s1[k], s0[k]
        for u, v in zip(a if isinstance(a, tuple) else (a,), b if isinstance(b, tuple) else (b,)):
            assert torch.equal(u, v), f"saved {k} differs"


def test_first_fuse_trainer_step_is_bitwise(cuda, monkeypatch):
    """The benchmarked step (c2, B = 256) with and without the fused first block: loss values
    and every gradient bitwise equal."""
    m = _model(cuda, 128, 16)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    x = torch.from_numpy(synthetic_patterns(3, 256)).to(cuda)
    eps = torch.from_numpy(seeded_eps(3, 256)).to(cuda)
    out = {}
    for fuse in (True, False):
        monkeypatch.setattr(E, "_FIRST_FUSE", "1" if fuse else "0")
        m.load_state_dict(sd)
        tr = VAETrainer(m, kl_lambda=5e-6)
        loss = tr.forward_backward(x, eps)
        torch.cuda.synchronize()
        out[fuse] = (torch.stack(loss).cpu(), tr.gflat.cpu())
    assert torch.equal(out[True][0], out[False][0])
    assert torch.equal(out[True][1], out[False][1])


def test_first_fuse_encode_latents(cuda, monkeypatch):
    """c4's path (encode_latents: the first conv statistics-only, y0 never written) gives the
    latents of the unfused path bit for bit."""
    m = _model(cuda, 128, 16)
    params = dict(m.named_parameters())
    x = torch.from_numpy(synthetic_patterns(5, 64)).to(cuda)
    mu = {}
    for fuse in (True, False):
        monkeypatch.setattr(E, "_FIRST_FUSE", "eval" if fuse else "0")
        with torch.no_grad():
            mu[fuse] = E.encode_latents(m.plan, x, params).cpu()
    assert torch.equal(mu[True], mu[False])
