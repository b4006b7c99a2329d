"""Fused Adam / AMSGrad on the HIP path (torch.optim.Adam semantics).

Drop-in for the reference's optimiser factories (latice/lightning_module.py:26-28:
`Adam(lr=1e-4, weight_decay=0, amsgrad=True)`; Hydra default
conf/lightning_module/default.yaml:10-13: `Adam(lr=1e-4)`).  One ebsdvae_adam launch per
parameter tensor (or per flat buffer, see trainer.FlatParams), state kept on the device,
bias corrections computed on the device from a device step counter.
"""
from __future__ import annotations

import torch

from . import _native as N
from . import engine as E


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 amsgrad=False):
        if lr < 0 or eps < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("invalid Adam hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                      amsgrad=amsgrad))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        E.before_weights_write()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients")
                st = self.state[p]
                if not st:
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    if group["amsgrad"]:
                        st["max_exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                if not p.is_contiguous():
                    raise RuntimeError("FusedAdam needs contiguous parameters")
                N.call("ebsdvae_adam", N.ptr(p), N.ptr(g), N.ptr(st["exp_avg"]),
                       N.ptr(st["exp_avg_sq"]), N.ptr(st.get("max_exp_avg_sq")), N.ptr(st["step"]),
                       p.numel(), float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                       float(group["weight_decay"]), int(bool(group["amsgrad"])), N.stream())
        E.weights_written()
        return loss
