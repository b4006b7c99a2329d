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


def test_deferred_tensor_computes_on_first_use_only():
    """latice.deferred.DeferredTensor (the eval/no-grad x_hat): metadata without running
    the thunk; any value access runs it once; results are plain tensors."""
    from latice.deferred import DeferredTensor
    calls = []

    def thunk():
        calls.append(1)
        return torch.arange(6.0).reshape(2, 1, 3)

    d = DeferredTensor(thunk, (2, 1, 3), torch.float32, torch.device("cpu"))
    assert d.shape == (2, 1, 3) and d.dim() == 3 and d.dtype == torch.float32 and len(d) == 2
    assert d.numel() == 6 and not d.requires_grad and not d.materialized and calls == []
    assert type(d * 2) is torch.Tensor and float((d * 2).sum()) == 30.0
    assert d.numpy().tolist() == [[[0.0, 1.0, 2.0]], [[3.0, 4.0, 5.0]]]
    assert torch.equal(torch.sigmoid(d), torch.sigmoid(torch.arange(6.0).reshape(2, 1, 3)))
    assert calls == [1] and d.materialized
    bad = DeferredTensor(lambda: torch.zeros(3), (2,), torch.float32, torch.device("cpu"))
    with pytest.raises(RuntimeError, match="does not match"):
        bad.sum()


def test_weight_writer_leaves_stale_deferred_values_to_their_reader():
    """engine.before_weights_write (run by every raw-pointer weight writer) computes the pending
    deferred values; one that can no longer be computed raises where it is read, not in the
    optimizer step that happened to flush it."""
    from latice import engine as E
    from latice.deferred import DeferredTensor, StaleDeferredError

    def stale():
        raise StaleDeferredError("model parameters changed between model(x) and the first use")

    good = DeferredTensor(lambda: torch.ones(2), (2,), torch.float32, torch.device("cpu"))
    bad = DeferredTensor(stale, (2,), torch.float32, torch.device("cpu"))
    E.defer_until_weights_change(bad)
    E.defer_until_weights_change(good)
    E.before_weights_write()            # does not raise
    assert good.materialized and not bad.materialized and not E._PENDING
    with pytest.raises(StaleDeferredError, match="parameters changed"):
        bad.sum()


def test_weight_writer_propagates_other_deferred_failures():
    """Only the stale case is left to the reader: any other failure while flushing a
    deferred value (a launch error, out of memory) propagates from the weight writer, before the
    weights change, and the value stays computable afterwards."""
    from latice import engine as E
    from latice.deferred import DeferredTensor

    calls = []

    def flaky():
        calls.append(1)
        if len(calls) == 1:
            raise RuntimeError("ebsdvae_conv3x3_fwd_split_st failed (1): out of memory")
        return torch.full((2,), 3.0)

    d = DeferredTensor(flaky, (2,), torch.float32, torch.device("cpu"))
    E.defer_until_weights_change(d)
    with pytest.raises(RuntimeError, match="out of memory"):
        E.before_weights_write()
    assert not d.materialized
    assert float(d.sum()) == 6.0 and d.materialized


def test_datamodule_split_matches_random_split(tmp_path):
    """DPDataModule.setup('fit') splits exactly like the reference's random_split with the
    seeded generator (latice/data_module.py:194-207); loaders report len() in batches."""
    import numpy as np
    from latice.data_module import DPDataModule
    np.save(tmp_path / "p.npy", np.zeros((23, 130, 130)))
    with open(tmp_path / "a.txt", "w") as f:
        f.write("eu\n23\n" + "".join(f"{i} {i} {i}\n" for i in range(23)))
    dm = DPDataModule(tmp_path / "p.npy", tmp_path / "a.txt", batch_size=4, val_data_ratio=0.25, seed=7)
    dm.setup("fit")
    perm = torch.randperm(23, generator=torch.Generator().manual_seed(7)).tolist()
    assert list(dm.dataset_train.indices) == perm[:18] and list(dm.dataset_val.indices) == perm[18:]
    assert len(dm.train_dataloader()) == 5 and len(dm.val_dataloader()) == 2
    assert list(dm.dataset_full.rot_angles.columns) == ["z1", "x", "z2"]
