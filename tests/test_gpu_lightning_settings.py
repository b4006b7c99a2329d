"""The drop-in under the reference's own trainer settings.

* `python train.py` trains with `precision: 16-mixed` (/root/reference/conf/train.yaml:14,
  conf/trainer/default.yaml:4): Lightning wraps the step in
  `torch.autocast("cuda", torch.float16)` and scales the loss with a GradScaler
  (x65536 at start).  The HIP path computes in its own fixed arithmetic whatever autocast
  says, so a x65536 gradient must flow through the per-image power-of-two f16 gradient
  scaling without overflow and, once unscaled, be the fixture's gradient (decision-pinned
  <= 1e-3, tests/pinned.py).
* Lightning 2.x runs `validation_step` (/root/reference/latice/lightning_module.py:296-346)
  in `model.eval()` under `torch.inference_mode()`: the model then returns x_hat deferred
  (latice/deferred.py) and the loss materialises it; values must be the fixture's.
"""
import numpy as np
import pytest
import torch

import latice.model as LM
from pinned import check_grads, fixture, host
from latice import engine as E
from latice.deferred import DeferredTensor
from latice.lightning_module import VAELightningModule, VAELoss
from latice.model import VariationalAutoEncoderRawData
from oracle import vae_oracle as O

pytestmark = pytest.mark.gpu


def _model(name, device):
    f, sd = fixture(name)
    B, S, L, ws, xs = (int(v) for v in f["meta"])
    m = VariationalAutoEncoderRawData(32, L, S)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return f, m.to(device)


@pytest.mark.parametrize("prec", ["f16x3", "fp32"])
def test_autocast_fp16_gradscaler_step(cuda, prec):
    f, m = _model("vae128_b4", cuda)
    x = torch.from_numpy(f["x"]).to(cuda)
    eps = torch.from_numpy(f["eps"]).to(cuda)
    opt = torch.optim.SGD(m.parameters(), lr=0.0)      # unscale_ needs an optimizer
    scaler = torch.amp.GradScaler("cuda", init_scale=65536.0)
    with E.precision(prec):
        with torch.autocast("cuda", dtype=torch.float16):
            with E.record_state() as rec:
                z, x_hat, mu, std = m(x, eps=eps)
            losses = VAELoss(kl_lambda=float(f["kl_lambda"])).compute_loss(z, x_hat, mu, std, x)
        assert losses["loss"].dtype == torch.float32 and x_hat.dtype == torch.float32
        scaler.scale(losses["loss"]).backward()
        scaler.unscale_(opt)
        torch.cuda.synchronize()
    found_inf = sum(float(v) for v in scaler._found_inf_per_device(opt).values())
    assert found_inf == 0.0, "a x65536-scaled gradient overflowed"
    ref = float(f["loss"])
    assert abs(float(losses["loss"]) - ref) <= 1e-5 * abs(ref)
    assert O.rel_err(host(x_hat), f["x_hat"]) < 1e-4
    grads = {n: p.grad for n, p in m.named_parameters()}
    check_grads("vae128_b4", m.plan, rec, grads, label=f"autocast-f16 + GradScaler {prec}", prec=prec)


def test_validation_step_under_inference_mode(cuda, monkeypatch):
    f, m = _model("vae128_b4", cuda)
    eps = torch.from_numpy(f["eps"]).to(cuda)
    # the reparameterisation noise of the step: the fixture's (model.forward draws it)
    monkeypatch.setattr(LM, "_draw_eps", lambda shape, device: eps.clone())
    module = VAELightningModule(m, kl_lambda=float(f["kl_lambda"]))
    module.eval()
    x = torch.from_numpy(f["x"]).to(cuda)
    angles = torch.zeros(x.shape[0], 3, dtype=torch.float64)
    with torch.inference_mode():
        z, x_hat, mu, std = m(x)
        assert isinstance(x_hat, DeferredTensor) and not x_hat.materialized
        metrics = module.validation_step((x, angles), 0)
        torch.cuda.synchronize()
    for k, key in (("loss", "val_loss"), ("kl_loss", "val_kl_loss"), ("recon_loss", "val_recon_loss")):
        ref = float(f[k])
        err = abs(float(metrics[key]) - ref) / abs(ref)
        print(f"\n{key}: rel err {err:.2e}")
        assert err <= 1e-5, key
    xh = metrics["x_hat"]
    assert isinstance(xh, DeferredTensor) and xh.materialized    # the loss read it
    assert O.rel_err(host(xh), f["x_hat"]) < 1e-4
    assert O.rel_err(host(metrics["x"]), f["x"]) == 0.0
    # the epoch hook stacks the detached step outputs (figure logging is out of scope)
    module.on_validation_epoch_end()
    assert np.isfinite(float(metrics["val_loss"]))
