"""The encoder-only fast path INSIDE model(x) and the unmodified build_dictionary flow on
the device (BASELINE c4), plus the drop-in DPDataModule loaders.

* model.eval() + no_grad: model(x) returns (z, x_hat, mu, std) with x_hat deferred; the call
  itself launches only encoder convs, mu/std/z equal the training forward's, and reading
  x_hat runs the decoder and gives the training forward's x_hat.
* DiffractionPatternIndexer.build_dictionary over a .npy + angle file: one model call per
  batch (tests/index/test_dp_indexer.py:305 in the reference), latents equal encode_mu of
  the on-device transform of the same patterns, orientations in file order.
"""
import numpy as np
import pytest
import torch

from latice import engine as E
from latice.data_module import DPDataModule, create_default_transform, ingest_patterns
from latice.deferred import DeferredTensor
from latice.index.dp_indexer import DiffractionPatternIndexer, IndexerConfig
from latice.model import VariationalAutoEncoderRawData
from latice.seeding import seeded_eps, seeded_state_dict, synthetic_patterns
from oracle import index_oracle as IO

pytestmark = pytest.mark.gpu


def _model(cuda):
    m = VariationalAutoEncoderRawData()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in seeded_state_dict(0).items()})
    return m.to(cuda)


def test_inference_forward_defers_the_decoder(cuda):
    m = _model(cuda)
    x = torch.from_numpy(synthetic_patterns(5, 6)).to(cuda)
    eps = torch.from_numpy(seeded_eps(5, 6)).to(cuda)
    with torch.no_grad():
        z_t, xh_t, mu_t, std_t = m(x, eps=eps)     # training mode: eager decoder
    m.eval()
    with torch.no_grad():
        with E.record_launches() as launched:
            z, x_hat, mu, std = m(x, eps=eps)
        assert isinstance(x_hat, DeferredTensor) and not x_hat.materialized
        assert x_hat.shape == (6, 1, 128, 128) and x_hat.dtype == torch.float32 and x_hat.is_cuda
        n_enc = len(launched)
        assert n_enc == len(m.plan.enc)       # the encoder's convs, nothing of the decoder
        # the inference path takes the first block's statistics from x's moments in double
        # (ebsdvae_conv_first_stats), the training-mode forward from its fp32 two-pass sums:
        # the two agree to rounding, not bit for bit
        def rel(a, b):
            return float((a - b).abs().max() / b.abs().max())
        for a, b in ((mu, mu_t), (std, std_t), (z, z_t)):
            assert rel(a, b) < 2e-5
        with E.record_launches() as launched:
            xh = x_hat.detach().cpu()
        assert len(launched) > 0 and x_hat.materialized
        assert rel(xh, xh_t.cpu()) < 5e-5
        # the deferred value behaves as a tensor in the reference's consumers
        assert torch.allclose(torch.sigmoid(x_hat), torch.sigmoid(xh_t), atol=5e-5)
        assert np.allclose(x_hat.cpu().numpy(), xh_t.cpu().numpy(), rtol=5e-5, atol=5e-5)
    # encode_mu is the same computation
    assert torch.allclose(m.encode_mu(x), mu, rtol=0, atol=1e-6)


def test_deferred_value_refuses_stale_weights(cuda):
    m = _model(cuda).eval()
    x = torch.from_numpy(synthetic_patterns(2, 2)).to(cuda)
    with torch.no_grad():
        _, x_hat, _, _ = m(x)
        m.decoder[14].bias.add_(1.0)
    with pytest.raises(RuntimeError, match="parameters changed"):
        x_hat.sum()


def _write_dataset(tmp_path, n, side, seed):
    rng = np.random.default_rng(seed)
    raw = rng.random((n, side, side))
    np.save(tmp_path / "patterns.npy", raw)
    ang = rng.uniform(0, 360, (n, 3)).round(3)
    with open(tmp_path / "angles.txt", "w") as f:
        f.write(f"eu\n{n}\n")
        for a in ang:
            f.write(f"{a[0]} {a[1]}  {a[2]}\n")
    return raw, ang


def test_build_dictionary_end_to_end(cuda, tmp_path):
    raw, ang = _write_dataset(tmp_path, 37, 140, 3)
    m = _model(cuda)
    calls = []
    m.register_forward_hook(lambda *a: calls.append(1))
    cfg = IndexerConfig(pattern_path=tmp_path / "patterns.npy", angles_path=tmp_path / "angles.txt",
                        batch_size=16, device="cuda")
    ix = DiffractionPatternIndexer(m, config=cfg)
    ix.build_dictionary()
    assert len(calls) == 3                      # ceil(37 / 16) batches, one call each
    assert ix.db.get_count() == 37
    assert np.allclose(ix.db.orientations, ang)
    x = ingest_patterns(raw, (128, 128))
    assert np.array_equal(x.cpu().numpy(), IO.ingest_patterns(raw))
    mu = m.encode_mu(x)
    lv = ix.db._db[:37]                         # the dictionary holds L2-normalised rows
    ref = torch.nn.functional.normalize(mu, dim=1)
    assert torch.allclose(lv, ref, atol=1e-5)
    # encode / index paths of the reference API
    e1 = ix.encode_pattern(raw[5])
    assert e1.shape == (16,) and np.allclose(e1, mu[5].cpu().numpy(), atol=1e-5)
    eb = ix.encode_patterns_batch(raw[:20])
    assert eb.shape == (20, 16) and np.allclose(eb, mu[:20].cpu().numpy(), atol=1e-5)
    res = ix.index_patterns_batch(raw[:4], top_n=5)
    assert len(res) == 4
    for j, r in enumerate(res):   # a pattern from the dictionary finds itself first
        assert np.allclose(r.candidate_orientations[0], ang[j])


def test_datamodule_loaders(cuda, tmp_path):
    raw, ang = _write_dataset(tmp_path, 50, 132, 4)
    dm = DPDataModule(tmp_path / "patterns.npy", tmp_path / "angles.txt", batch_size=8,
                      val_data_ratio=0.2, seed=42)
    dm.setup("fit")
    assert len(dm.dataset_train) == 40 and len(dm.dataset_val) == 10
    ref_perm = torch.randperm(50, generator=torch.Generator().manual_seed(42)).tolist()
    assert list(dm.dataset_train.indices) == ref_perm[:40]   # torch random_split semantics
    ref_x = IO.ingest_patterns(raw)
    seen = []
    tl = dm.train_dataloader()
    assert len(tl) == 5
    for x, a in tl:
        assert x.is_cuda and x.shape[1:] == (1, 128, 128) and a.dtype == torch.float64
        rows = [int(np.flatnonzero((ang == r.numpy()).all(1))[0]) for r in a]
        assert np.array_equal(x.cpu().numpy(), ref_x[rows])
        seen += rows
    assert sorted(seen) == sorted(ref_perm[:40])
    dm.setup("test")
    got = torch.cat([x for x, _ in dm.test_dataloader()]).cpu().numpy()
    assert np.array_equal(got, ref_x)
    t = create_default_transform((128, 128))
    assert np.array_equal(t(raw[3]).cpu().numpy(), ref_x[3])


def test_deferred_value_survives_a_fused_optimizer_step(cuda):
    """A pending x_hat is computed with the weights of the model(x) call that made it, even
    when a fused Adam step (raw-pointer writes) runs before it is read, and when it is read
    on another stream."""
    from latice.optim import FusedAdam
    m = _model(cuda)
    x = torch.from_numpy(synthetic_patterns(4, 2)).to(cuda)
    eps = torch.from_numpy(seeded_eps(4, 2)).to(cuda)
    m.eval()
    with torch.no_grad():
        _, ref, _, _ = m(x, eps=eps)
        ref = ref.detach().clone()
        _, x_hat, _, _ = m(x, eps=eps)
    assert not x_hat.materialized
    opt = FusedAdam(m.parameters(), lr=1e-2)
    for p in m.parameters():
        p.grad = torch.ones_like(p)
    opt.step()                                   # materialises x_hat first
    assert x_hat.materialized
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        got = x_hat.detach().clone()
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    with torch.no_grad():                        # the new weights do change the output
        _, x2, _, _ = m(x, eps=eps)
        assert not torch.equal(x2.detach(), ref)
