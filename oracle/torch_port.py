"""ORACLE (test / baseline infrastructure only) — PyTorch-CPU restatement of the
reference training step, used as bench.py's `cpu_baseline` ("port").

Functional form of latice/model.py:40-150 (conv/convT -> InstanceNorm2d -> LeakyReLU,
MaxPool2d, UpsamplingNearest2d, Linear heads, reparameterisation) and
latice/lightning_module.py:79-156 (BCE-with-logits + MC KL), differentiated by torch
autograd on the CPU and followed by torch.optim.Adam, i.e. what the reference's
training_step costs on the host cores.  The reference source itself never leaves the
survey container; parity of this port is pinned in tests/test_torch_port.py against the
same golden vectors as the numpy oracle.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

ENC_IDX = (0, 1, 3, 4, 6, 7, 9, 10, 12, 13)
DEC_IDX = (1, 2, 4, 5, 7, 8, 10, 11, 13)


def forward(p: dict, x: torch.Tensor, eps: torch.Tensor):
    a = x
    for i, idx in enumerate(ENC_IDX):
        a = F.conv2d(a, p[f"encoder.{idx}.0.weight"], p[f"encoder.{idx}.0.bias"], padding=1)
        a = F.leaky_relu(F.instance_norm(a, eps=1e-5), 0.02)
        if i % 2 == 1:
            a = F.max_pool2d(a, 2, 2)
    enc = a
    flat = enc.flatten(1, -1)
    mu = F.linear(flat, p["mu.0.weight"], p["mu.0.bias"])
    logvar = F.linear(flat, p["logvar.0.weight"], p["logvar.0.bias"])
    std = torch.exp(logvar / 2)
    z = mu + eps * torch.exp(logvar / 2)
    a = F.linear(z, p["linear2.0.weight"], p["linear2.0.bias"]).view(enc.size())
    for i, idx in enumerate(DEC_IDX):
        if i % 2 == 0:
            a = F.interpolate(a, scale_factor=2, mode="nearest")
        a = F.conv_transpose2d(a, p[f"decoder.{idx}.0.weight"], p[f"decoder.{idx}.0.bias"], padding=1)
        a = F.leaky_relu(F.instance_norm(a, eps=1e-5), 0.02)
    x_hat = F.conv2d(a, p["decoder.14.weight"], p["decoder.14.bias"], padding=1)
    return z, x_hat, mu, std


def loss(z, x_hat, mu, std, x, kl_lambda: float):
    recon = F.binary_cross_entropy_with_logits(x_hat, x, reduction="none").mean(dim=(1, 2, 3))
    q = torch.distributions.Normal(mu, std)
    pz = torch.distributions.Normal(torch.zeros_like(mu), torch.ones_like(std))
    kl = (q.log_prob(z) - pz.log_prob(z)).mean(-1) * kl_lambda
    elbo = kl + recon
    return {"loss": elbo.mean(), "kl_loss": kl.mean(), "recon_loss": recon.mean(), "elbo": elbo}


class CPUStep:
    """fwd + loss + bwd + Adam(lr 1e-4) on the CPU (the cpu_baseline workload)."""

    def __init__(self, state_dict: dict, kl_lambda: float = 5e-6, lr: float = 1e-4):
        self.p = {k: torch.as_tensor(v).clone().float().requires_grad_(True)
                  for k, v in state_dict.items()}
        self.opt = torch.optim.Adam(self.p.values(), lr=lr)
        self.kl_lambda = kl_lambda

    def step(self, x: torch.Tensor, eps: torch.Tensor) -> float:
        self.opt.zero_grad(set_to_none=True)
        z, x_hat, mu, std = forward(self.p, x, eps)
        out = loss(z, x_hat, mu, std, x, self.kl_lambda)
        out["loss"].backward()
        self.opt.step()
        return float(out["loss"].detach())

    @torch.no_grad()
    def encode(self, x: torch.Tensor) -> torch.Tensor:
        """Encoder + mu head (what build_dictionary keeps, latice/index/dp_indexer.py:284-287)."""
        a = x
        for i, idx in enumerate(ENC_IDX):
            a = F.conv2d(a, self.p[f"encoder.{idx}.0.weight"], self.p[f"encoder.{idx}.0.bias"], padding=1)
            a = F.leaky_relu(F.instance_norm(a, eps=1e-5), 0.02)
            if i % 2 == 1:
                a = F.max_pool2d(a, 2, 2)
        return F.linear(a.flatten(1, -1), self.p["mu.0.weight"], self.p["mu.0.bias"])
