"""Drop-in API surface of latice.model / latice.lightning_module (CPU: construction,
state_dict compatibility, plan topology, and the no-CPU-fallback guarantee)."""
import numpy as np
import pytest
import torch

from latice import engine as E
from latice.lightning_module import (VAELightningModule, VAELoss, get_default_optimiser,
                                     get_default_scheduler)
from latice.model import VariationalAutoEncoder, VariationalAutoEncoderRawData
from latice.seeding import layer_table, seeded_state_dict

REF_KEYS = [r[0] for r in layer_table()]


def test_state_dict_keys_and_shapes_match_reference():
    m = VariationalAutoEncoderRawData()
    sd = m.state_dict()
    assert list(sd.keys()) == REF_KEYS          # the 46 keys of latice/model.py
    for name, shape, _ in layer_table():
        assert tuple(sd[name].shape) == shape, name
    assert sum(p.numel() for p in m.parameters()) == 1_853_793


def test_256_variant_param_count():
    m = VariationalAutoEncoderRawData(inplanes=32, latent_dim=64, image_size=256)
    assert sum(p.numel() for p in m.parameters()) == 3_334_593


def test_default_init_is_torch_default_like_reference():
    """Same module classes in the same order => identical default init under a seed."""
    torch.manual_seed(123)
    a = VariationalAutoEncoderRawData().state_dict()
    torch.manual_seed(123)
    b = VariationalAutoEncoderRawData().state_dict()
    for k in a:
        assert torch.equal(a[k], b[k])
    # conv weight std ~0.034 (kaiming-uniform), not 0.02: weights_init is a no-op
    assert 0.025 < float(a["encoder.1.0.weight"].std()) < 0.045


def test_load_seeded_state_dict_roundtrip():
    m = VariationalAutoEncoderRawData()
    sd = {k: torch.from_numpy(v) for k, v in seeded_state_dict(0).items()}
    m.load_state_dict(sd)
    assert torch.equal(m.encoder[3][0].weight, sd["encoder.3.0.weight"])
    assert isinstance(m, VariationalAutoEncoder)
    assert callable(m.encoder) and callable(m.mu) and callable(m.decoder)


def test_no_cpu_fallback():
    m = VariationalAutoEncoderRawData()
    with pytest.raises(RuntimeError, match="ROCm device|libebsdvae"):
        m(torch.rand(2, 1, 128, 128))


def test_plan_topology():
    p = E.build_plan()
    assert [L.H for L in p.enc] == [128, 128, 64, 64, 32, 32, 16, 16, 8, 8]
    assert [L.H for L in p.dec] == [8, 8, 16, 16, 32, 32, 64, 64, 128]
    assert [L.src_mode for L in p.enc] == [0, 1, 2, 1, 2, 1, 2, 1, 2, 1]
    assert [L.pmode for L in p.enc] == [0, 1, 0, 1, 0, 1, 0, 1, 0, 1]
    assert [L.src_mode for L in p.dec] == [3, 1, 4, 1, 4, 1, 4, 1, 4]
    assert [L.pmode for L in p.dec] == [0, 2, 0, 2, 0, 2, 0, 2, 0]
    names = {L.name + ".weight" for L in p.enc + p.dec}
    assert names <= set(REF_KEYS)
    assert p.feat == 2048 and E.build_plan(32, 64, 256).feat == 8192


def test_lightning_module_api():
    m = VariationalAutoEncoderRawData()
    lm = VAELightningModule(m, kl_lambda=5e-6)
    assert isinstance(lm.loss_fn, VAELoss) and lm.loss_fn.kl_lambda == 5e-6
    opt = get_default_optimiser(m.parameters())
    assert opt.defaults["amsgrad"] is True and opt.defaults["lr"] == 1e-4
    sched = get_default_scheduler(opt)   # the reference's factory raises on torch 2.10
    assert sched is not None
    cfg = lm.configure_optimizers()
    assert set(cfg) == {"optimizer", "lr_scheduler", "monitor"}
