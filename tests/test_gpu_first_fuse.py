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
    # the staging itself: inference's statistics from the first conv's fma chain, as the
    # unfused path computes them (the moment-based ones: test_first_fuse_encode_latents)
    monkeypatch.setattr(E, "_FIRST_GRAM", False)
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


@pytest.mark.parametrize("gram", [False, True], ids=["fma-stats", "gram-stats"])
def test_first_fuse_encode_latents(cuda, monkeypatch, gram):
    """c4's path (encode_latents: the first conv statistics-only, y0 never written) against the
    unfused path: bit for bit when the statistics come from the first conv's own fma chain
    (EBSDVAE_FIRST_GRAM=0); with the default moment-based statistics (ebsdvae_conv_first_stats,
    double) the {mean, rstd} differ from the fp32 two-pass ones by rounding only, and so do the
    latents."""
    monkeypatch.setattr(E, "_FIRST_GRAM", gram)
    m = _model(cuda, 128, 16)
    params = dict(m.named_parameters())
    x = torch.from_numpy(synthetic_patterns(5, 64)).to(cuda)
    mu = {}
    for fuse in (True, False):
        monkeypatch.setattr(E, "_FIRST_FUSE", "eval" if fuse else "0")
        with torch.no_grad():
            mu[fuse] = E.encode_latents(m.plan, x, params).cpu()
    if not gram:
        assert torch.equal(mu[True], mu[False])
    else:
        err = float((mu[True] - mu[False]).abs().max() / mu[False].abs().max())
        print(f"\nlatents, moment-based vs two-pass first-conv statistics: {err:.2e}")
        assert err < 2e-5


@pytest.mark.parametrize("S,B", [(128, 64), (256, 4), (128, 3)])
def test_first_conv_stats_from_moments(cuda, S, B):
    """ebsdvae_conv_first_stats (the 9 shifted means and 45 second moments of x, double) against
    the first conv's own two-pass statistics (ebsdvae_conv_first_fwd + finalize) and the float64
    oracle."""
    import numpy as np
    from oracle import vae_oracle as O
    m = _model(cuda, S, 16 if S == 128 else 64)
    L0 = m.plan.enc[0]
    w, b = m.encoder[0][0].weight, m.encoder[0][0].bias
    x = torch.from_numpy(synthetic_patterns(2, B, S)).to(cuda)
    st = torch.empty(B, 32, 2, device=cuda)
    from latice import _native as N
    N.call("ebsdvae_conv_first_stats", N.ptr(x), N.ptr(w), N.ptr(b), N.ptr(st), B, S, S, 32, N.stream())
    _, st_ref = E._conv_first(x, L0, w, b, B, write_y=True)
    torch.cuda.synchronize()
    y64 = O.conv3x3(x.double().cpu().numpy().transpose(0, 2, 3, 1),
                    w.double().detach().cpu().numpy(), b.double().detach().cpu().numpy())
    mean = y64.mean(axis=(1, 2))
    rstd = 1.0 / np.sqrt(y64.var(axis=(1, 2)) + 1e-5)
    got = st.double().cpu().numpy()
    two = st_ref.double().cpu().numpy()
    e_mean = np.abs(got[..., 0] - mean).max() / np.abs(mean).max()
    e_rstd = np.abs(got[..., 1] - rstd).max() / np.abs(rstd).max()
    e_two = np.abs(two[..., 1] - rstd).max() / np.abs(rstd).max()
    print(f"\nmoments: mean {e_mean:.2e} rstd {e_rstd:.2e} (two-pass fp32 rstd {e_two:.2e})")
    assert e_mean < 1e-6 and e_rstd < 1e-6
