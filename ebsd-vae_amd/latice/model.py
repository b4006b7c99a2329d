"""Drop-in `latice.model` (reference: latice/model.py) running on MI355X HIP kernels.

Same classes, constructor arguments, submodule names, parameter shapes, default init and
46-key state_dict as the reference, so `load_state_dict(torch.load("vae-best.pt"))`,
Hydra `_target_: latice.model.VariationalAutoEncoderRawData`, `model(x)[2]`,
`model.encoder(x)`, `model.mu(...)`, `model.reparameterize(...)` all keep working.

What changes is what runs: the `encoder` / `decoder` containers and the latent heads
execute the fused HIP path of engine.py (libebsdvae.so) instead of module-by-module
ATen ops.  The inner building blocks stay ordinary torch modules purely as parameter
holders (identical init and state_dict); they are not on the hot path.  There is no CPU
fallback: the model must live on a ROCm device (model.to("cuda")).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from . import engine as E
from .deferred import DeferredTensor, StaleDeferredError
from .functional import DecoderFn, EncoderFn, HeadsFn, LinearFn, ReparamFn

# EBSDVAE_DEFER_DECODE=0: the eval/no-grad forward runs the decoder eagerly (A/B timing)
_DEFER = os.environ.get("EBSDVAE_DEFER_DECODE", "1") != "0"


def _draw_eps(shape, device) -> torch.Tensor:
    """N(0,1) noise from the HIP Philox sampler, seeded from torch's (CPU) generator so that
    torch.manual_seed(...) makes runs reproducible (replaces Normal.rsample's normal_)."""
    eps = torch.empty(shape, dtype=torch.float32, device=device)
    seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    return E.normal_(eps, seed)


class HipLinear(nn.Linear):
    """nn.Linear whose forward runs the HIP linear kernel (same init / state_dict)."""

    def forward(self, x):
        return LinearFn.apply(x, self.weight, self.bias)


class _FusedEncoder(nn.Sequential):
    """`model.encoder` (latice/model.py:109-125): calling it runs the fused HIP encoder."""

    def __init__(self, plan, *mods):
        super().__init__(*mods)
        object.__setattr__(self, "_plan", plan)

    def _params(self):
        out = []
        for L in self._plan.enc:
            conv = self[int(L.name.split(".")[1])][0]
            out += [conv.weight, conv.bias]
        return out

    def forward(self, x):
        return EncoderFn.apply(self._plan, x, *self._params())


class _FusedDecoder(nn.Sequential):
    """`model.decoder` (latice/model.py:133-150): calling it runs the fused HIP decoder."""

    def __init__(self, plan, *mods):
        super().__init__(*mods)
        object.__setattr__(self, "_plan", plan)

    def _params(self):
        out = []
        for L in self._plan.dec:
            conv = self[int(L.name.split(".")[1])][0]
            out += [conv.weight, conv.bias]
        return out + [self[14].weight, self[14].bias]

    def forward(self, x):
        return DecoderFn.apply(self._plan, x, *self._params())


class VariationalAutoEncoder(nn.Module):
    """Base class (latice/model.py:7-80): reparameterisation + forward."""

    def __init__(self) -> None:
        super().__init__()
        self.apply(self.weights_init)   # a no-op here exactly as in the reference (:16)
        self.encoder = None
        self.mu = None
        self.logvar = None
        self.linear2 = None
        self.decoder = None

    def reparameterize(self, mu: torch.Tensor, logvar: torch.Tensor) -> torch.Tensor:
        """z ~ N(mu, exp(logvar/2)) via z = mu + eps*std, eps from the HIP sampler."""
        return ReparamFn.apply(mu, logvar, _draw_eps(mu.shape, mu.device))

    def forward(self, x: torch.Tensor, eps: torch.Tensor | None = None):
        """Returns (z, x_hat, mu, std) like latice/model.py:40-66.  `eps` (B, latent) may be
        supplied to make the reparameterisation noise deterministic (parity tests).

        In eval mode with autograd off (build_dictionary, encode_pattern(s), validation)
        x_hat comes back as a DeferredTensor: the decoder runs only if x_hat is used, so
        `_, _, mu, _ = model(data)` (latice/index/dp_indexer.py:136,183,284) costs the
        encoder and the heads alone -- one model call per batch, as the reference's callers
        and tests expect (tests/index/test_dp_indexer.py:305)."""
        if _DEFER and not self.training and not torch.is_grad_enabled():
            return self._forward_inference(x, eps)
        enc = self.encoder(x)
        if eps is None:
            eps = _draw_eps((x.shape[0], self.mu[0].out_features), x.device)
        z, mu, std, dec_in = HeadsFn.apply(
            self._plan, enc, eps, self.mu[0].weight, self.mu[0].bias, self.logvar[0].weight,
            self.logvar[0].bias, self.linear2[0].weight, self.linear2[0].bias)
        x_hat = self.decoder(dec_in)
        return z, x_hat, mu, std

    def _inference_packs(self, params):
        """Packed conv weights for inference launches, repacked only when a parameter changed
        (storage or version counter) or the conv arithmetic was switched."""
        key = (E.get_precision(), E.weights_generation()) + tuple(
            (p.data_ptr(), p._version) for p in params.values())
        cached = getattr(self, "_packcache", None)
        if cached is None or cached[0] != key:
            ps = E.PackSet(self._plan, params)
            cached = (key, ps, ps.refresh())
            object.__setattr__(self, "_packcache", cached)
        return cached[2]

    def _forward_inference(self, x, eps):
        if x.device.type != "cuda":
            raise RuntimeError("the HIP VAE needs a ROCm device tensor (no CPU fallback)")
        plan = self._plan
        x = x.float().contiguous()
        params = dict(self.named_parameters())
        packs = self._inference_packs(params)
        enc, _ = E.encoder_forward(plan, x, params, packs=packs, train=False)
        if eps is None:
            eps = _draw_eps((x.shape[0], plan.latent_dim), x.device)
        _, mu, std, z, dec_in = E.heads_forward(plan, enc, params, eps.float().contiguous())
        versions = [(p, p._version) for p in params.values()]
        gen = E.weights_generation()
        # the decoder may run later on another stream: it waits for this point of the stream
        # that made dec_in (and the packs)
        made_on = torch.cuda.current_stream(x.device)
        ready = torch.cuda.Event()
        ready.record(made_on)

        def decode():
            # raw-pointer weight writers materialise pending values first
            # (engine.before_weights_write); a torch in-place update bumps _version
            if gen != E.weights_generation() or any(p._version != v for p, v in versions):
                raise StaleDeferredError("model parameters changed between model(x) and the first "
                                         "use of its deferred x_hat")
            cur = torch.cuda.current_stream(x.device)
            if cur != made_on:
                cur.wait_event(ready)
                dec_in.record_stream(cur)
            with torch.no_grad():
                x_hat, _ = E.decoder_forward(plan, dec_in, params,
                                             packs=self._inference_packs(params))
            return x_hat

        S = plan.image_size
        x_hat = DeferredTensor(decode, (x.shape[0], 1, S, S), torch.float32, x.device)
        E.defer_until_weights_change(x_hat)
        return z, x_hat, mu, std

    @torch.no_grad()
    def encode_mu(self, x: torch.Tensor) -> torch.Tensor:
        """Encoder-only fast path: mu == forward(x)[2] (the only output
        DiffractionPatternIndexer.build_dictionary keeps, latice/index/dp_indexer.py:136),
        without the reparameterisation and decoder."""
        if x.device.type != "cuda":
            raise RuntimeError("encode_mu needs a ROCm device tensor (no CPU fallback)")
        params = dict(self.named_parameters())
        return E.encode_latents(self._plan, x.float().contiguous(), params,
                                packs=self._inference_packs(params))

    @staticmethod
    def weights_init(m: nn.Module) -> None:
        """Kept for API parity with latice/model.py:68-80."""
        classname = m.__class__.__name__
        if classname.find("Conv") != -1:
            m.weight.data.normal_(0.0, 0.02)
        elif classname.find("BatchNorm") != -1:
            m.weight.data.normal_(1.0, 0.02)
            m.bias.data.fill_(0)


class VariationalAutoEncoderRawData(VariationalAutoEncoder):
    """latice/model.py:83-150.  `image_size` (default 128, the reference's only working
    size) also allows the 256x256 variant of BASELINE config 5 (heads of width
    4*inplanes*(image_size/32)^2)."""

    def __init__(self, inplanes: int = 32, latent_dim: int = 16, image_size: int = 128):
        super().__init__()
        plan = E.build_plan(inplanes, latent_dim, image_size)
        object.__setattr__(self, "_plan", plan)

        def building_blocks(in_dim, out_dim, filter_size=3, stride=1, padding=1):
            return nn.Sequential(
                nn.Conv2d(in_dim, out_dim, filter_size, stride=stride, padding=padding),
                nn.InstanceNorm2d(out_dim),
                nn.LeakyReLU(0.02),
            )

        def building_blocks_trans(in_dim, out_dim, filter_size=3, stride=1, padding=1):
            return nn.Sequential(
                nn.ConvTranspose2d(in_dim, out_dim, filter_size, stride=stride, padding=padding),
                nn.InstanceNorm2d(out_dim),
                nn.LeakyReLU(0.02),
            )

        p = inplanes
        self.encoder = _FusedEncoder(
            plan,
            building_blocks(1, p), building_blocks(p, p), nn.MaxPool2d(2, 2),
            building_blocks(p, 2 * p), building_blocks(2 * p, 2 * p), nn.MaxPool2d(2, 2),
            building_blocks(2 * p, 4 * p), building_blocks(4 * p, 4 * p), nn.MaxPool2d(2, 2),
            building_blocks(4 * p, 4 * p), building_blocks(4 * p, 4 * p), nn.MaxPool2d(2, 2),
            building_blocks(4 * p, 4 * p), building_blocks(4 * p, 4 * p), nn.MaxPool2d(2, 2),
        )
        feat = plan.feat
        self.mu = nn.Sequential(HipLinear(feat, latent_dim))
        self.logvar = nn.Sequential(HipLinear(feat, latent_dim))
        self.linear2 = nn.Sequential(HipLinear(latent_dim, feat))
        self.decoder = _FusedDecoder(
            plan,
            nn.UpsamplingNearest2d(scale_factor=2),
            building_blocks_trans(4 * p, 4 * p), building_blocks_trans(4 * p, 4 * p),
            nn.UpsamplingNearest2d(scale_factor=2),
            building_blocks_trans(4 * p, 4 * p), building_blocks_trans(4 * p, 4 * p),
            nn.UpsamplingNearest2d(scale_factor=2),
            building_blocks_trans(4 * p, 4 * p), building_blocks_trans(4 * p, 2 * p),
            nn.UpsamplingNearest2d(scale_factor=2),
            building_blocks_trans(2 * p, 2 * p), building_blocks_trans(2 * p, p),
            nn.UpsamplingNearest2d(scale_factor=2),
            building_blocks_trans(p, p),
            nn.Conv2d(p, 1, 3, 1, 1),
        )

    @property
    def plan(self):
        return self._plan
