"""Drop-in `latice.lightning_module` (reference: latice/lightning_module.py).

`VAELoss.compute_loss` runs the fused HIP BCE + Monte-Carlo KL kernels (forward and
backward, functional.VAELossFn); `VAELightningModule` keeps the reference's constructor,
`_get_step_outputs`, `training_step` (returns {"loss": ...}), `validation_step`,
`test_step`, epoch hooks and `configure_optimizers`.  pytorch_lightning is optional:
when it is importable the module subclasses `pl.LightningModule`, otherwise a plain
`nn.Module` with a no-op `log` so the step logic can still be driven directly.
"""
from __future__ import annotations

import inspect
import math
from typing import Any, Protocol

import torch
from torch import nn
from torch.optim import Optimizer

from .functional import KLFn, VAELossFn
from .model import VariationalAutoEncoder
from .optim import FusedAdam

try:  # pragma: no cover - depends on the environment
    import pytorch_lightning as pl
    _Base = pl.LightningModule
    HAVE_LIGHTNING = True
except Exception:  # noqa: BLE001
    pl = None
    HAVE_LIGHTNING = False

    class _Base(nn.Module):
        """Minimal stand-in when pytorch_lightning is absent."""

        current_epoch = 0
        logger = None

        def log(self, *args, **kwargs):
            return None


class OptimizerPartial(Protocol):
    def __call__(self, params: Any) -> Optimizer:
        raise NotImplementedError


class SchedulerPartial(Protocol):
    def __call__(self, optimizer: Optimizer) -> Any:
        raise NotImplementedError


def get_default_optimiser(params: Any) -> Optimizer:
    """latice/lightning_module.py:26-28: Adam(lr=1e-4, weight_decay=0, amsgrad=True),
    here as the fused HIP Adam with identical update rule."""
    return FusedAdam(params=params, lr=1e-4, weight_decay=0, amsgrad=True)


def get_default_scheduler(optimizer: Optimizer) -> Any:
    """latice/lightning_module.py:31-35.  torch >= 2.8 removed ReduceLROnPlateau's
    `verbose` argument (the reference call raises TypeError there); pass it only where
    it still exists."""
    kw = dict(factor=0.1, patience=10)
    if "verbose" in inspect.signature(torch.optim.lr_scheduler.ReduceLROnPlateau).parameters:
        kw["verbose"] = True
    return torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, **kw)


class VAELoss:
    """latice/lightning_module.py:38-156."""

    def __init__(self, kl_lambda: float = 0.1):
        self.kl_lambda = kl_lambda
        self.log_scale = nn.Parameter(torch.Tensor([0.0]))

    def gaussian_likelihood(self, x_hat, logscale, x):
        """Unused by the reference's training path (:53-77); kept for API completeness."""
        scale = torch.exp(logscale)
        dist = torch.distributions.Normal(x_hat, scale)
        log_pxz = dist.log_prob(x)
        log_pxz = log_pxz + torch.log(torch.sqrt(torch.tensor(2 * math.pi)) * scale)
        return log_pxz.mean(dim=(1, 2, 3))

    def _fused(self, z, x_hat, mu, std, x):
        return VAELossFn.apply(z, x_hat, mu, std, x, float(self.kl_lambda))

    def binary_cross_entropy(self, x_hat, x):
        """Per-sample mean BCE-with-logits (:79-92), via the fused kernel with lambda = 0."""
        B = x_hat.shape[0]
        zeros = torch.zeros(B, 1, device=x_hat.device, dtype=torch.float32)
        ones = torch.ones(B, 1, device=x_hat.device, dtype=torch.float32)
        *_, elbo = VAELossFn.apply(zeros, x_hat, zeros, ones, x, 0.0)
        return elbo

    def kl_divergence(self, z, mu, std):
        """Per-sample MC KL (:94-120) (unscaled): the loss kernel's own kl_b at lambda = 1."""
        return KLFn.apply(z, mu, std)

    def compute_loss(self, z, x_hat, mu, std, x) -> dict[str, torch.Tensor]:
        """:122-156 -> {"loss", "kl_loss", "recon_loss", "elbo"}; kl_loss is already x lambda."""
        loss, kl_loss, recon_loss, elbo = self._fused(z, x_hat, mu, std, x)
        return {"loss": loss, "kl_loss": kl_loss, "recon_loss": recon_loss, "elbo": elbo}


class VAELightningModule(_Base):
    """latice/lightning_module.py:159-369."""

    def __init__(self, model: VariationalAutoEncoder, kl_lambda: float = 0.1,
                 optimizer_partial: OptimizerPartial = get_default_optimiser,
                 lr_scheduler_partial: SchedulerPartial = get_default_scheduler) -> None:
        super().__init__()
        self.model = model
        self.loss_fn = VAELoss(kl_lambda=kl_lambda)
        self.optimizer_partial = optimizer_partial
        self.lr_scheduler_partial = lr_scheduler_partial
        self.latent = []
        self._set_random_seeds()
        self.validation_step_outputs = []
        self.training_step_outputs = []

    def _set_random_seeds(self, seed: int = 42) -> None:
        torch.manual_seed(seed)
        torch.cuda.manual_seed_all(seed)

    def forward(self, x):
        return self.model(x)

    def _get_step_outputs(self, batch, prefix: str = ""):
        x, _ = batch
        z, x_hat, mu, std = self(x)
        losses = self.loss_fn.compute_loss(z, x_hat, mu, std, x)
        metrics = {
            f"{prefix}loss": losses["loss"],
            f"{prefix}kl_loss": losses["kl_loss"],
            f"{prefix}recon_loss": losses["recon_loss"],
        }
        if prefix == "val_":
            metrics["x"] = x
            metrics["x_hat"] = x_hat
        return metrics

    def training_step(self, train_batch, batch_idx: int):
        metrics = self._get_step_outputs(train_batch, prefix="train_")
        # the reference keeps graph-attached tensors for the whole epoch (:263, a leak);
        # store detached scalars with the same keys instead
        self.training_step_outputs.append({k: v.detach() for k, v in metrics.items()})
        self.log("elbo", metrics["train_loss"], prog_bar=True, on_step=True)
        self.log("train_kl_loss", metrics["train_kl_loss"], prog_bar=True, on_step=True)
        self.log("train_recon_loss", metrics["train_recon_loss"], prog_bar=True, on_step=True)
        return {"loss": metrics["train_loss"]}

    def on_train_epoch_end(self) -> None:
        outs = self.training_step_outputs
        if outs:
            for key, name in (("train_loss", "Epoch_train_loss"),
                              ("train_kl_loss", "Epoch_train_kl_loss"),
                              ("train_recon_loss", "Epoch_train_recon_loss")):
                self.log(name, torch.stack([o[key] for o in outs]).mean())
        self.training_step_outputs = []

    def validation_step(self, val_batch, batch_idx: int):
        metrics = self._get_step_outputs(val_batch, prefix="val_")
        self.validation_step_outputs.append({k: v.detach() for k, v in metrics.items()})
        self.log("val_loss", metrics["val_loss"], prog_bar=True, on_step=True)
        self.log("val_kl_loss", metrics["val_kl_loss"], prog_bar=True, on_step=True)
        self.log("val_recon_loss", metrics["val_recon_loss"], prog_bar=True, on_step=True)
        return metrics

    def on_validation_epoch_end(self) -> None:
        outs = self.validation_step_outputs
        if outs:
            for key, name in (("val_loss", "Epoch_val_loss"), ("val_kl_loss", "Epoch_val_kl_loss"),
                              ("val_recon_loss", "Epoch_val_recon_loss")):
                self.log(name, torch.stack([o[key] for o in outs]).mean())
        # figure logging (plot_detection / log_fig, :331-343) is visualisation, out of scope
        self.validation_step_outputs = []

    def test_step(self, test_batch, batch_idx: int):
        x, _ = test_batch
        _, _, embeddings, _ = self(x)
        return embeddings

    def test_epoch_end(self, test_step_outputs) -> None:
        embeddings = torch.cat([x for x in test_step_outputs], dim=0)
        self.latent = embeddings.detach().cpu().numpy()

    def configure_optimizers(self):
        optimizer = self.optimizer_partial(self.model.parameters())
        if self.lr_scheduler_partial:
            scheduler = self.lr_scheduler_partial(optimizer)
            return {"optimizer": optimizer, "lr_scheduler": scheduler, "monitor": "val_loss"}
        return optimizer
