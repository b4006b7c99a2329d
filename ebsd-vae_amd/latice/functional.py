"""torch.autograd wrappers over the HIP engine (the drop-in autograd surface).

Each Function's forward/backward is a fixed sequence of libebsdvae.so launches
(engine.py); no ATen compute op runs on the hot path.  Activations cross the Python
boundary as NCHW-shaped tensors with channels_last (== NHWC) memory, so callers see the
reference's shapes while the kernels read NHWC without a transpose.
"""
from __future__ import annotations

import torch

from . import engine as E
from . import _native as N


def _nhwc(t):
    """NCHW-shaped tensor -> (B,H,W,C) contiguous view (copy only if not channels_last)."""
    return t.permute(0, 2, 3, 1).contiguous()


def _nchw_view(t):
    """(B,H,W,C) contiguous -> NCHW-shaped channels_last view."""
    return t.permute(0, 3, 1, 2)


def _f32c(t):
    if t is None:
        return None
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


def enc_param_names(plan):
    return [L.name + s for L in plan.enc for s in (".weight", ".bias")]


def dec_param_names(plan):
    return [L.name + s for L in plan.dec for s in (".weight", ".bias")] + [
        "decoder.14.weight", "decoder.14.bias"]


class EncoderFn(torch.autograd.Function):
    """x (B,1,S,S) -> encoder output (B,4p,S/32,S/32); latice/model.py:109-125."""

    @staticmethod
    def forward(ctx, plan, x, *params):
        names = enc_param_names(plan)
        pd = dict(zip(names, params))
        x = _f32c(x)
        out, saved = E.encoder_forward(plan, x, pd)
        ctx.plan, ctx.names, ctx.acts = plan, names, saved
        ctx.save_for_backward(x, *params)
        ctx.set_materialize_grads(False)
        return _nchw_view(out)

    @staticmethod
    def backward(ctx, g):
        x, *params = ctx.saved_tensors
        if g is None:
            return (None, None) + (None,) * len(params)
        pd = dict(zip(ctx.names, params))
        grads, gx = E.encoder_backward(ctx.plan, _nhwc(_f32c(g)), x, ctx.acts, pd,
                                       need_gx=ctx.needs_input_grad[1])
        ctx.acts = None
        return (None, gx) + tuple(grads[n] for n in ctx.names)


class HeadsFn(torch.autograd.Function):
    """enc (B,C,s,s) -> (z, mu, std, dec_in (B,C,s,s)); latice/model.py:55-64 + :25-38."""

    @staticmethod
    def forward(ctx, plan, enc, eps, *params):
        pd = dict(zip(E.HEAD_NAMES, params))
        flat, mu, std, z, dec_in = E.heads_forward(plan, _nhwc(_f32c(enc)), pd, _f32c(eps))
        ctx.plan = plan
        ctx.save_for_backward(flat, std, z, eps, *params)
        ctx.set_materialize_grads(False)
        return z, mu, std, _nchw_view(dec_in)

    @staticmethod
    def backward(ctx, g_z, g_mu, g_std, g_dec):
        flat, std, z, eps, *params = ctx.saved_tensors
        pd = dict(zip(E.HEAD_NAMES, params))
        B = z.shape[0]
        plan = ctx.plan
        if g_dec is None:
            g_dec_t = torch.zeros(B, plan.enc_side, plan.enc_side, plan.enc_channels,
                                  device=z.device, dtype=torch.float32)
        else:
            g_dec_t = _nhwc(_f32c(g_dec))
        g_enc, grads = E.heads_backward(plan, g_dec_t, _f32c(g_z), _f32c(g_mu), _f32c(g_std), flat,
                                        std, z, _f32c(eps), pd)
        return (None, _nchw_view(g_enc), None) + tuple(grads[n] for n in E.HEAD_NAMES)


class DecoderFn(torch.autograd.Function):
    """dec_in (B,C,s,s) -> x_hat logits (B,1,S,S); latice/model.py:133-150."""

    @staticmethod
    def forward(ctx, plan, dec_in, *params):
        names = dec_param_names(plan)
        pd = dict(zip(names, params))
        x_hat, saved = E.decoder_forward(plan, _nhwc(_f32c(dec_in)), pd)
        ctx.plan, ctx.names, ctx.acts = plan, names, saved
        ctx.save_for_backward(*params)
        ctx.set_materialize_grads(False)
        return x_hat

    @staticmethod
    def backward(ctx, g):
        params = ctx.saved_tensors
        if g is None:
            return (None, None) + (None,) * len(params)
        pd = dict(zip(ctx.names, params))
        grads, g_dec = E.decoder_backward(ctx.plan, _f32c(g), ctx.acts, pd)
        ctx.acts = None
        return (None, _nchw_view(g_dec)) + tuple(grads[n] for n in ctx.names)


class VAELossFn(torch.autograd.Function):
    """(z, x_hat, mu, std, x) -> (loss, kl_loss, recon_loss, elbo); lightning_module.py:122-156."""

    @staticmethod
    def forward(ctx, z, x_hat, mu, std, x, kl_lambda):
        z, x_hat, mu, std, x = (_f32c(t) for t in (z, x_hat, mu, std, x))
        (loss, kl_loss, recon_loss), (elbo, _, _) = E.loss_forward(x_hat, x, z, mu, std, kl_lambda)
        ctx.kl_lambda = float(kl_lambda)
        ctx.save_for_backward(z, x_hat, mu, std, x)
        ctx.set_materialize_grads(False)
        return loss, kl_loss, recon_loss, elbo

    @staticmethod
    def backward(ctx, g_loss, g_kl, g_recon, g_elbo):
        z, x_hat, mu, std, x = ctx.saved_tensors
        g_xhat, g_z, g_mu, g_std, g_x = E.loss_backward(
            x_hat, x, z, mu, std, ctx.kl_lambda, _f32c(g_loss), _f32c(g_kl), _f32c(g_recon),
            _f32c(g_elbo), need_gx=ctx.needs_input_grad[4])
        return g_z, g_xhat, g_mu, g_std, g_x, None


class KLFn(torch.autograd.Function):
    """(z, mu, std) -> per-sample Monte-Carlo KL, unscaled (lightning_module.py:94-120):
    mean_j [log N(z; mu, std) - log N(z; 0, 1)], read directly from the loss kernel's kl_b
    output at lambda = 1 with an all-zero BCE partial (ebsdvae_vae_loss_fwd_parts), so no
    reconstruction term is added and subtracted again."""

    @staticmethod
    def forward(ctx, z, mu, std):
        z, mu, std = (_f32c(t) for t in (z, mu, std))
        B = z.shape[0]
        end = E.NetEnd(None, None, None, None, torch.zeros(B, 1, device=z.device), 1)
        _, (_, kl, _) = E.loss_forward_parts(end, z, mu, std, 1.0, 1)
        ctx.save_for_backward(z, mu, std)
        return kl

    @staticmethod
    def backward(ctx, g):
        z, mu, std = ctx.saved_tensors
        # d kl_b / d(z, mu, std) == d elbo_b / d(z, mu, std) when there is no x_hat
        _, g_z, g_mu, g_std, _ = E.loss_backward(None, None, z, mu, std, 1.0, g_elbo=_f32c(g), P=1)
        return g_z, g_mu, g_std


class LinearFn(torch.autograd.Function):
    """nn.Linear on the HIP path (direct calls of model.mu / .logvar / .linear2)."""

    @staticmethod
    def forward(ctx, x, w, b):
        x2 = _f32c(x).reshape(-1, x.shape[-1])
        M, K = x2.shape
        Nn = w.shape[0]
        y = torch.empty(M, Nn, device=x.device, dtype=torch.float32)
        N.call("ebsdvae_linear_fwd", N.ptr(x2), N.ptr(w), N.ptr(b), N.ptr(y), M, K, Nn, N.stream())
        ctx.save_for_backward(x2, w, b)
        ctx.in_shape = x.shape
        return y.reshape(*x.shape[:-1], Nn)

    @staticmethod
    def backward(ctx, gy):
        x2, w, b = ctx.saved_tensors
        M, K = x2.shape
        Nn = w.shape[0]
        gy2 = _f32c(gy).reshape(M, Nn)
        gx = torch.empty_like(x2) if ctx.needs_input_grad[0] else None
        gw = torch.empty_like(w) if ctx.needs_input_grad[1] else None
        gb = torch.empty_like(b) if (b is not None and ctx.needs_input_grad[2]) else None
        N.call("ebsdvae_linear_bwd", N.ptr(x2), N.ptr(w), N.ptr(gy2), N.ptr(gx), N.ptr(gw), N.ptr(gb),
               M, K, Nn, N.stream())
        return (gx.reshape(ctx.in_shape) if gx is not None else None), gw, gb


class ReparamFn(torch.autograd.Function):
    """z = mu + eps * exp(logvar/2) (latice/model.py:25-38) with supplied eps."""

    @staticmethod
    def forward(ctx, mu, logvar, eps):
        mu, logvar, eps = _f32c(mu), _f32c(logvar), _f32c(eps)
        z = torch.empty_like(mu)
        std = torch.empty_like(mu)
        N.call("ebsdvae_reparam_fwd", N.ptr(mu), N.ptr(logvar), N.ptr(eps), N.ptr(z), N.ptr(std),
               mu.numel(), N.stream())
        ctx.save_for_backward(eps, std)
        return z

    @staticmethod
    def backward(ctx, gz):
        eps, std = ctx.saved_tensors
        gmu = torch.empty_like(std)
        glv = torch.empty_like(std)
        N.call("ebsdvae_reparam_bwd", N.ptr(_f32c(gz)), None, N.ptr(eps), N.ptr(std), N.ptr(gmu),
               N.ptr(glv), std.numel(), N.stream())
        return gmu, glv, None
