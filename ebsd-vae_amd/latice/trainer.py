"""Training-step driver for the MI355X path: the work of
`VAELightningModule.training_step` + `loss.backward()` + `optimizer.step()`
(latice/lightning_module.py:248-273, :359-369) without autograd bookkeeping, and the
data-parallel version of it that the reference only gets implicitly from Lightning DDP.

* Parameters are re-pointed into ONE flat fp32 buffer and gradients are written by the
  kernels straight into ONE flat gradient buffer (ordered decoder -> heads -> encoder, the
  order in which the backward finishes them), so the optimiser is a single fused Adam
  launch and the gradient exchange is two contiguous RCCL all-reduces.
* Data parallelism (one process per GPU, torch.distributed "nccl" == RCCL over xGMI):
  every rank processes its own batch shard; the loss gradient is pre-scaled by 1/W so a
  SUM all-reduce yields the mean gradient with no extra pass.  Three buckets, in the order
  the backward completes them: 0 = decoder + heads (3.6 MB at 128x128, started after the
  heads backward), 1 = the deep encoder layers at <= S/4 resolution (3.2 MB, started once
  their weight gradients are issued, beside the shallow encoder backward), 2 = the shallow
  encoder layers (0.26 MB, the only all-reduce left after the backward).  7.4 MB per step in
  total (1.85M fp32 parameters); DESIGN.md section 6 gives the expected exposed time.
* N == 1: the whole step can be captured into a hipGraph (capture()/replay()).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _native as N
from . import engine as E
from .functional import dec_param_names, enc_param_names


class GradReducer:
    """Bucketed asynchronous SUM all-reduce of a flat gradient buffer: `split` is one bucket
    boundary (two buckets) or an increasing sequence of them."""

    def __init__(self, gflat: torch.Tensor, split, group=None, force: bool = False):
        """force: issue the all-reduces even in a group of one rank (tests run the collective
        path -- side-stream issue, wait ordering -- on a single GPU)."""
        cuts = [int(split)] if isinstance(split, int) else [int(c) for c in split]
        self.bounds = [0] + cuts + [gflat.numel()]
        if any(b > c for b, c in zip(self.bounds, self.bounds[1:])):
            raise ValueError(f"bucket boundaries must increase within the buffer: {self.bounds}")
        self.gflat, self.split, self.group = gflat, cuts[0], group
        inited = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if inited else 1
        if force and not inited:
            raise RuntimeError("GradReducer(force=True) needs an initialised process group")
        self.active = self.world > 1 or bool(force)
        self._works = []

    def start(self, bucket: int):
        if not self.active:
            return
        t = self.gflat[self.bounds[bucket]:self.bounds[bucket + 1]]
        if t.numel() == 0:
            return
        self._works.append(dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def finish(self):
        for w in self._works:
            w.wait()
        self._works = []


def shard_batch(x: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    """Contiguous 1/W slice of a global batch."""
    B = x.shape[0]
    if B % world:
        raise ValueError(f"global batch {B} not divisible by world size {world}")
    per = B // world
    return x[rank * per:(rank + 1) * per]


class VAETrainer:
    def __init__(self, model, kl_lambda: float = 5e-6, lr: float = 1e-4, betas=(0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0, amsgrad: bool = False,
                 seed: int = 0, group=None, force_allreduce: bool = False):
        self.model = model
        self.plan = model.plan
        self.kl_lambda = float(kl_lambda)
        self.lr, self.betas, self.adam_eps = float(lr), betas, float(eps)
        self.weight_decay, self.amsgrad = float(weight_decay), bool(amsgrad)
        self.seed = int(seed)
        params = dict(model.named_parameters())
        dev = next(iter(params.values())).device
        if dev.type != "cuda":
            raise RuntimeError("VAETrainer needs the model on a ROCm device (no CPU fallback)")
        dec = dec_param_names(self.plan) + list(E.HEAD_NAMES)
        # encoder parameters in the order the backward finishes them: the deep layers (at most
        # S/4 resolution, 93 % of the encoder's parameters) first, then the shallow ones
        S = self.plan.image_size
        deep = [L for L in reversed(self.plan.enc) if L.H <= S // 4]
        shallow = [L for L in reversed(self.plan.enc) if L.H > S // 4]
        enc = [L.name + s for L in deep + shallow for s in (".weight", ".bias")]
        if sorted(enc) != sorted(enc_param_names(self.plan)):
            raise RuntimeError("unexpected encoder parameter set")
        # the all-reduce of bucket 1 starts once the last deep layer's weight gradient is issued
        self._deep_last = deep[-1].name if deep and shallow else None
        order = dec + enc
        if set(order) != set(params):
            raise RuntimeError("unexpected parameter set")
        total = sum(params[n].numel() for n in order)
        self.flat = torch.empty(total, device=dev, dtype=torch.float32)
        self.gflat = torch.zeros(total, device=dev, dtype=torch.float32)
        self.P, self.G = {}, {}
        off = 0
        with torch.no_grad():
            for n in order:
                p = params[n]
                k = p.numel()
                view = self.flat[off:off + k].view_as(p)
                view.copy_(p.data)
                p.data = view
                self.P[n] = p
                self.G[n] = self.gflat[off:off + k].view_as(p)
                off += k
        self.split = sum(params[n].numel() for n in dec)
        n_deep = sum(params[L.name + s].numel() for L in deep for s in (".weight", ".bias"))
        self.buckets = [self.split, self.split + n_deep] if self._deep_last else [self.split]
        self.exp_avg = torch.zeros_like(self.flat)
        self.exp_avg_sq = torch.zeros_like(self.flat)
        self.max_exp_avg_sq = torch.zeros_like(self.flat) if self.amsgrad else None
        self.step_count = torch.zeros((), device=dev, dtype=torch.float32)
        self.one = torch.ones((), device=dev, dtype=torch.float32)
        self.noise_counter = torch.zeros(1, device=dev, dtype=torch.int64)
        self.reducer = GradReducer(self.gflat, self.buckets, group, force=force_allreduce)
        self.world = self.reducer.world
        if self.world > 1:
            # every rank starts from rank 0's parameters (broadcast once
            # at init; Lightning DDP does the same when it wraps the model)
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast(self.flat, src=src, group=group)
        self._eps = None
        # bench.py (N > 1): events around the gradient exchange's exposed tail
        self.time_allreduce = False
        self.allreduce_events = []
        self.graph = None
        self._static = None
        self.packset = E.PackSet(self.plan, self.P)   # params are views of self.flat

    @property
    def numel(self) -> int:
        return self.flat.numel()

    def _noise(self, B):
        L = self.plan.latent_dim
        if self._eps is None or self._eps.shape[0] != B:
            self._eps = torch.empty(B, L, device=self.flat.device, dtype=torch.float32)
        return E.normal_(self._eps, self.seed, counter=self.noise_counter)

    def forward_backward(self, x: torch.Tensor, eps: torch.Tensor | None = None):
        """fwd + loss + bwd into self.gflat (+ the DP gradient exchange).  Returns the three
        loss scalars (device tensors)."""
        plan, P, G = self.plan, self.P, self.G
        if E.poisoned():   # debug: every gradient element must be written by this step
            self.gflat.fill_(float("nan"))
        # one launch packs every conv weight of the step, and the reparameterisation noise is
        # drawn: both on the side stream, beside the first conv (which reads its weight
        # unpacked); the current stream waits for them before the first packed layer
        side = E.side_stream(x.device) if E.side_streams_enabled() else None
        if side is not None:
            main = torch.cuda.current_stream(x.device)
            E.stream_wait(side, main)
            with torch.cuda.stream(side):
                packs = self.packset.refresh()
                eps = self._noise(x.shape[0]) if eps is None else eps
            ready = lambda: E.stream_wait(main, side)   # noqa: E731
        else:
            packs = self.packset.refresh()
            eps = self._noise(x.shape[0]) if eps is None else eps
            ready = None
        enc, se = E.encoder_forward(plan, x, P, packs=packs, packs_ready=ready)
        flat, mu, std, z, dec_in = E.heads_forward(plan, enc, P, eps)
        fused_end = E.net_end_ok(plan)
        x_hat, sd = E.decoder_forward(plan, dec_in, P, packs=packs, final=not fused_end)
        # the side stream (weight gradients, their slice reductions, the heads' weight
        # gradients, the loss values) is joined once, after the encoder backward: only the
        # chain loss backward -> input gradients -> ... stays on the current stream
        with E.deferred_side_join(x.device):
            if fused_end:
                # final conv + BCE + its logit gradient + the last block's reduce: one pass
                x_hat, end = E.network_end(plan, sd, P, x, g_loss=self.one, scale=1.0 / self.world)
                (loss, kl, rec), _ = E.loss_forward_parts(end, z, mu, std, self.kl_lambda,
                                                          x[0].numel())
                _, g_z, g_mu, g_std, _ = E.loss_backward(None, None, z, mu, std, self.kl_lambda,
                                                         g_loss=self.one, scale=1.0 / self.world,
                                                         P=x[0].numel())
                _, g_dec = E.decoder_backward(plan, None, sd, P, grads=G, packs=packs, end=end)
            else:
                (loss, kl, rec), _ = E.loss_forward(x_hat, x, z, mu, std, self.kl_lambda)
                g_xhat, g_z, g_mu, g_std, _ = E.loss_backward(x_hat, x, z, mu, std, self.kl_lambda,
                                                              g_loss=self.one,
                                                              scale=1.0 / self.world)
                _, g_dec = E.decoder_backward(plan, g_xhat, sd, P, grads=G, packs=packs)
            g_enc, _ = E.heads_backward(plan, g_dec, g_z, g_mu, g_std, flat, std, z, eps, P,
                                        grads=G)
            hooks = {}
            if self.reducer.active:
                # bucket 0 (decoder + heads) is complete on the side stream once it has
                # caught up with the heads backward: the all-reduce is ordered behind it
                self._start_behind_side(0, x.device)
                if self._deep_last:
                    hooks[self._deep_last] = lambda: self._start_behind_side(1, x.device)
            E.encoder_backward(plan, g_enc, x, se, P, grads=G, packs=packs, after_wgrad=hooks)
        ev = None
        if self.time_allreduce and self.reducer.active:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()   # the backward (both streams, joined above) is done here
        self.reducer.start(len(self.reducer.bounds) - 2)   # the last bucket
        self.reducer.finish()
        if ev is not None:
            ev[1].record()   # ... and every bucket's all-reduce here
            self.allreduce_events.append(ev)
        return loss, kl, rec

    def allreduce_exposed_ms(self):
        """Mean GPU time per timed step between the end of the backward and the completion of
        the last all-reduce (the part of the gradient exchange no backward work hides), over
        the steps run with time_allreduce set; None when no collective ran.  Synchronises."""
        if not self.allreduce_events:
            return None
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in self.allreduce_events]
        self.allreduce_events = []
        return sum(ms) / len(ms)

    def _start_behind_side(self, bucket: int, device):
        """Start a bucket's all-reduce behind everything issued so far on both streams: the
        side stream carries the weight gradients (and their reductions), the current stream
        the rest (heads backward, first-layer fused weight gradient)."""
        if not E.side_streams_enabled():
            self.reducer.start(bucket)
            return
        side = E.side_stream(device)
        E.stream_wait(side, torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            self.reducer.start(bucket)

    def optimizer_step(self):
        b1, b2 = self.betas
        E.before_weights_write()
        N.call("ebsdvae_adam", N.ptr(self.flat), N.ptr(self.gflat), N.ptr(self.exp_avg),
               N.ptr(self.exp_avg_sq), N.ptr(self.max_exp_avg_sq), N.ptr(self.step_count),
               self.flat.numel(), self.lr, float(b1), float(b2), self.adam_eps, self.weight_decay,
               int(self.amsgrad), N.stream())
        E.weights_written()

    def step(self, x: torch.Tensor, eps: torch.Tensor | None = None):
        out = self.forward_backward(x, eps)
        self.optimizer_step()
        return out

    # ------------------------------------------------------------------ hipGraph (N == 1)
    def capture(self, x: torch.Tensor, warmup: int = 1):
        """Capture one whole step on static input `x` (N == 1 only: collectives stay out
        of graphs).  Warm-up steps run first on a side stream, as torch requires."""
        if self.world != 1:
            raise RuntimeError("graph capture is for single-process runs")
        E.side_stream(x.device)   # the weight-gradient stream exists before the capture
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.step(x)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = self.step(x)
        self.graph, self._static = g, (x, out)
        return out

    def replay(self):
        E.before_weights_write()
        self.graph.replay()
        E.weights_written()
        return self._static[1]
