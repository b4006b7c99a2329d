"""Launch plan of the VAE hot path over the C ABI (no autograd here).

This module knows the network topology of `VariationalAutoEncoderRawData`
(latice/model.py:109-150 in the reference) and sequences the HIP kernels of
libebsdvae.so for the forward and the explicitly derived backward:

    encoder:  10 x [conv3x3 -> InstanceNorm -> LeakyReLU], MaxPool2d after every 2nd
    heads:    flatten(NCHW) -> mu / logvar -> std, z = mu + eps*std -> linear2 -> view
    decoder:  5 x [Upsample -> 2 x (convT3x3 -> InstanceNorm -> LeakyReLU)] -> conv3x3(32->1)
    loss:     BCE-with-logits + lambda * MC-KL     (latice/lightning_module.py:79-156)

Every activation is NHWC fp32.  Each conv block saves only its pre-norm output y and its
InstanceNorm statistics; all normalised / pooled / upsampled activations are recomputed
on the fly by the consuming kernel (forward, dgrad and wgrad alike).

All functions take and return torch tensors purely as device-memory handles; buffers come
from the PyTorch caching allocator and every launch goes to the current HIP stream.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import weakref
from dataclasses import dataclass, field

import torch

from . import _native as N

ACT_RAW, ACT_NORM, ACT_NORM_POOL, ACT_UP, ACT_NORM_UP = range(5)
P_ID, P_POOL, P_UP = range(3)
P_UPSUM = 3   # ebsdvae_conv3x3_dgrad_inbwd_split: P_UP with the 2x2-summed gradient as output
KIND_CONV, KIND_CONVT = 0, 1


@dataclass(frozen=True)
class ConvLayer:
    name: str       # parameter prefix, e.g. "encoder.3.0"
    kind: int       # KIND_CONV / KIND_CONVT
    cin: int
    cout: int
    H: int          # output (== logical input) spatial size
    src_mode: int   # how this conv reads its input
    pmode: int      # how the consumer reads THIS layer's output (for the IN backward)


@dataclass(frozen=True)
class Plan:
    inplanes: int
    latent_dim: int
    image_size: int
    enc: tuple = field(default=())
    dec: tuple = field(default=())

    @property
    def enc_channels(self) -> int:
        return 4 * self.inplanes

    @property
    def enc_side(self) -> int:
        return self.image_size // 32

    @property
    def feat(self) -> int:
        return self.enc_channels * self.enc_side ** 2


def build_plan(inplanes: int = 32, latent_dim: int = 16, image_size: int = 128) -> Plan:
    """Topology of latice/model.py:109-148 (encoder idx 0,1,3,4,...; decoder idx 1,2,4,...)."""
    p, S = inplanes, image_size
    if S % 32 or S < 64:
        raise ValueError(f"image_size must be a multiple of 32 and >= 64 (got {S})")
    enc_io = [(1, p), (p, p), (p, 2 * p), (2 * p, 2 * p), (2 * p, 4 * p), (4 * p, 4 * p),
              (4 * p, 4 * p), (4 * p, 4 * p), (4 * p, 4 * p), (4 * p, 4 * p)]
    enc_idx = (0, 1, 3, 4, 6, 7, 9, 10, 12, 13)
    enc = []
    for i, ((ci, co), idx) in enumerate(zip(enc_io, enc_idx)):
        H = S >> (i // 2)
        if i == 0:
            mode = ACT_RAW
        else:
            mode = ACT_NORM if i % 2 == 1 else ACT_NORM_POOL
        pmode = P_POOL if i % 2 == 1 else P_ID
        enc.append(ConvLayer(f"encoder.{idx}.0", KIND_CONV, ci, co, H, mode, pmode))
    dec_io = [(4 * p, 4 * p), (4 * p, 4 * p), (4 * p, 4 * p), (4 * p, 4 * p), (4 * p, 4 * p),
              (4 * p, 2 * p), (2 * p, 2 * p), (2 * p, p), (p, p)]
    dec_idx = (1, 2, 4, 5, 7, 8, 10, 11, 13)
    dec = []
    for i, ((ci, co), idx) in enumerate(zip(dec_io, dec_idx)):
        H = S >> (4 - i // 2)
        if i == 0:
            mode = ACT_UP
        else:
            mode = ACT_NORM if i % 2 == 1 else ACT_NORM_UP
        # consumer of this layer: next layer (or the final conv, which reads ACT_NORM)
        nxt = ACT_NORM if i == len(dec_io) - 1 else (ACT_NORM if (i + 1) % 2 == 1 else ACT_NORM_UP)
        pmode = P_UP if nxt == ACT_NORM_UP else P_ID
        dec.append(ConvLayer(f"decoder.{idx}.0", KIND_CONVT, ci, co, H, mode, pmode))
    return Plan(inplanes, latent_dim, image_size, tuple(enc), tuple(dec))


# ----------------------------------------------------------------------------- probes
_PROBE = None


class probe:
    """Record HIP events around the conv kernel launches (bench.py's live per-kernel
    timing): records (family, algorithmic_flops, ev_start, ev_end) on the current stream."""

    def __init__(self):
        self.records = []

    def __enter__(self):
        global _PROBE
        _PROBE = self.records
        return self

    def __exit__(self, *exc):
        global _PROBE
        _PROBE = None

    def per_tag(self):
        """{tag: [launches, flops, ms]} (per-layer view for tools/layer_profile.py)."""
        torch.cuda.synchronize()
        out = {}
        for fam, flops, e0, e1, tag, _, _ in self.records:
            d = out.setdefault(f"{fam} {tag}", [0, 0.0, 0.0])
            d[0] += 1
            d[1] += flops
            d[2] += e0.elapsed_time(e1)
        return out

    def attainable_s(self, hbm_bytes_per_s: float = 8e12) -> float:
        """Sum over the recorded launches of max(F_k / P_k, B_k / BW): the attainable-roofline
        time of these kernels, F_k the algorithmic fp32-equivalent
        FLOPs, P_k the peak of the launch's arithmetic, B_k its algorithmic I/O bytes."""
        return sum(max(flops / (mfma_peak(pieces) * 1e12), nb / hbm_bytes_per_s)
                   for _, flops, _, _, _, pieces, nb in self.records)

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for fam, flops, e0, e1, _, pieces, _ in self.records:
            d = out.setdefault(fam, {"launches": 0, "flops": 0.0, "ms": 0.0, "peak_s": 0.0,
                                     "split_launches": 0})
            d["launches"] += 1
            d["flops"] += flops
            d["ms"] += e0.elapsed_time(e1)
            d["peak_s"] += flops / (mfma_peak(pieces) * 1e12)   # time at this launch's peak
            d["split_launches"] += 1 if pieces else 0
        return out


FP32_MFMA_TFLOPS = 157.3    # MI355X dense peaks (MI355X_MICROARCH.md)
BF16_MFMA_TFLOPS = 2516.6


def mfma_peak(pieces: int) -> float:
    """Peak in fp32-equivalent TFLOP/s of a conv launch: fp32 MFMA, or the bf16 MFMA peak
    divided by the bf16 products per fp32 product of the split (3 or 6)."""
    return FP32_MFMA_TFLOPS if not pieces else BF16_MFMA_TFLOPS / {2: 3, 3: 6, PIECES_F16: 3}[pieces]


_LAUNCHES = None


@contextlib.contextmanager
def record_launches():
    """Test hook: the C-ABI entry points of the conv launches issued inside the block."""
    global _LAUNCHES
    outer, lst = _LAUNCHES, []
    _LAUNCHES = lst
    try:
        yield lst
    finally:
        _LAUNCHES = outer


def _launch(family, flops, fn, *args, tag=None, pieces=0, nbytes=0):
    if _LAUNCHES is not None:
        _LAUNCHES.append(args[0] if fn is N.call else getattr(fn, "__name__", str(fn)))
    if _PROBE is None:
        return fn(*args)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    r = fn(*args)
    e1.record()
    _PROBE.append((family, float(flops), e0, e1, tag, pieces, float(nbytes)))
    return r


def conv_flops(B, H, W, cin, cout):
    return 2.0 * B * H * W * cin * cout * 9


# ----------------------------------------------------------------------------- weight writes
# Kernels that update parameters through raw pointers (the fused Adam) bypass torch's
# version counters; they bump this generation so cached weight packs are refreshed.
_WEIGHTS_GEN = 0


def weights_written() -> None:
    global _WEIGHTS_GEN
    _WEIGHTS_GEN += 1


def weights_generation() -> int:
    return _WEIGHTS_GEN


# Deferred inference outputs (model.py: the decoder half of an eval/no-grad forward) that have
# not been read yet.  Every raw-pointer weight writer calls before_weights_write() first, so
# they are computed with the weights of the model(x) call that made them, as the reference
# would have returned them then.
_PENDING = {}   # id -> weakref (tensors compare elementwise, so no WeakSet)


def defer_until_weights_change(t) -> None:
    key = id(t)

    def gone(ref, key=key):
        if _PENDING.get(key) is ref:
            del _PENDING[key]
    _PENDING[key] = weakref.ref(t, gone)


def before_weights_write() -> None:
    """Materialise every pending deferred value (called before a fused optimizer step or a
    graph replay writes parameters through raw pointers).  A value that can no longer be
    computed (its parameters already changed through torch: StaleDeferredError) is left to
    raise where it is read, not here: the weight writer is not the call site at fault.  Any
    other failure (a launch error, out of memory) propagates from here, before the weights
    change.  Nothing runs while a stream is being captured (the decoder launches would land
    in the graph)."""
    from .deferred import StaleDeferredError
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        return
    while _PENDING:
        _, ref = _PENDING.popitem()
        t = ref()
        if t is not None:
            try:
                t.materialize()
            except StaleDeferredError:
                pass   # materialize() keeps the thunk: the first read raises the same error


# ----------------------------------------------------------------------------- state record
_RECORD = None


@contextlib.contextmanager
def record_state():
    """Test hook: collects {layer name: (y, st)} -- the pre-norm conv output and InstanceNorm
    statistics every conv block of a training forward saves for its backward -- of the
    forwards run inside the block (the decision/state-pinned oracle of the parity tests,
    oracle.vae_oracle.forward_from_state).  Holds references only; nothing is copied."""
    global _RECORD
    outer, rec = _RECORD, {}
    _RECORD = rec
    try:
        yield rec
    finally:
        _RECORD = outer


def _record(plan_layers, saved):
    if _RECORD is not None:
        _RECORD.update({L.name: saved[L.name] for L in plan_layers if L.name in saved})


# ----------------------------------------------------------------------------- helpers
# EBSDVAE_POISON=1 (debug): every buffer the engine hands to a kernel -- outputs, gradients,
# statistics / slice partials and scratch -- is NaN-filled when allocated, so a kernel that
# leaves any element of it unwritten, or a consumer that reads one before its producer wrote
# it, shows up as a NaN in the results (tests/test_gpu_poison.py).  set_poison() switches it.
_POISON = os.environ.get("EBSDVAE_POISON", "0") not in ("", "0")


def set_poison(on: bool) -> None:
    global _POISON
    _POISON = bool(on)


def poisoned() -> bool:
    return _POISON


def _scratch(*shape, dtype=torch.float32, device):
    if _POISON:
        return torch.full(shape, float("nan"), dtype=dtype, device=device)
    return torch.empty(shape, dtype=dtype, device=device)


def _empty(*shape, like):
    return _scratch(*shape, device=like.device)


def _empty_like(t):
    if _POISON:
        return torch.full_like(t, float("nan"))
    return torch.empty_like(t)


def _f64(*shape, device):
    return _scratch(*shape, dtype=torch.float64, device=device)


# ----------------------------------------------------------------------------- precision
# Conv arithmetic (csrc/conv_fwd.hip, csrc/conv_split.hip, csrc/conv_wgrad.hip):
#   "fp32"   v_mfma_f32_32x32x2_f32 (exact fp32 products);
#   "bf16x6" 3-piece split-bf16 MFMA, 6 products per fp32 product (~2^-25, fp32 grade);
#   "bf16x3" 2-piece split-bf16 MFMA, 3 products (~2^-16.5 per product);
#   "f16x3"  2-piece split-fp16 MFMA (x0 = f16(x), x1 = f16(x - x0)), 3 products (~2^-22.5
#            per product) for the forward, input-gradient and weight-gradient convs: weights
#            packed as w * 2^k with one power of two per layer from max |w| (pack trailer),
#            the gradient operand scaled by a power of two per image (input gradient) or per
#            slice (weight gradient) from the per-tile max |gy| the InstanceNorm-backward apply
#            emits; where a layer has no fp16 kernel (8x8 weight gradient of an upsampled
#            source) it takes bf16x6.
# Split modes cover every conv layer the split kernels support (Cout in {32,64,128},
# H*W >= 256, plus the 8x8 maps); the 1->32 first conv is an fp32 VALU kernel in every mode
# (ebsdvae_conv_first_fwd; EBSDVAE_FIRST_VALU=0: the fp32-MFMA kernel).
PIECES_F16 = 16   # EBSDVAE_PIECES_F16 (include/ebsdvae.h)
_PIECES = {"fp32": 0, "bf16x3": 2, "bf16x6": 3, "f16x3": 3}
_FWD_PIECES = {"f16x3": PIECES_F16}   # forward-conv piece format where it differs
# default: f16x3; passes every fp32 parity gate (tests/test_gpu_model.py and
# tests/test_gpu_trainer.py run fp32, bf16x6 and f16x3)
_PRECISION = os.environ.get("EBSDVAE_PRECISION", "f16x3")
if _PRECISION not in _PIECES:
    raise ValueError(f"EBSDVAE_PRECISION must be one of {sorted(_PIECES)}")
_SPLIT_CACHE = {}


def set_precision(mode: str):
    global _PRECISION
    if mode not in _PIECES:
        raise ValueError(f"precision must be one of {sorted(_PIECES)}, not {mode!r}")
    _PRECISION = mode


def get_precision() -> str:
    return _PRECISION


@contextlib.contextmanager
def precision(mode: str):
    """Temporarily switch the conv arithmetic (tests, A/B runs)."""
    old = _PRECISION
    set_precision(mode)
    try:
        yield
    finally:
        set_precision(old)


def _supported(H: int, cin: int, cout: int, np_: int) -> bool:
    key = (H, cin, cout, np_)
    if key not in _SPLIT_CACHE:
        _SPLIT_CACHE[key] = bool(N.call("ebsdvae_conv3x3_split_supported", H, H, cin, cout, np_))
    return _SPLIT_CACHE[key]


def split_pieces(H: int, cin: int, cout: int, dgrad: bool = False, scaled: bool = False) -> int:
    """Piece format of a conv with input channels cin -> cout at HxH: bf16 pieces per operand
    (2 or 3), PIECES_F16, or 0 = fp32.  dgrad: the input-gradient pack, fp16 only when its
    gradient operand comes with per-tile maxima (scaled: in_backward(..., gmax=True))."""
    np_ = _PIECES[_PRECISION]
    if np_ == 0:
        return 0
    f16 = _FWD_PIECES.get(_PRECISION)
    if f16 and (not dgrad or scaled) and _supported(H, cin, cout, f16):
        return f16
    return np_ if _supported(H, cin, cout, np_) else 0


@dataclass
class PackedW:
    t: torch.Tensor
    pieces: int   # 0 = fp32 pack


def _pack_numel(layer: ConvLayer, pieces: int, dgrad: bool) -> int:
    if not pieces:
        return 9 * layer.cin * layer.cout
    ci_, co_ = (layer.cout, layer.cin) if dgrad else (layer.cin, layer.cout)
    return N.call("ebsdvae_pack_split_bytes", ci_, co_, pieces) // 4


def pack_weight(w, layer: ConvLayer, dgrad: bool, scaled: bool = False) -> PackedW:
    """scaled: the input-gradient operand will carry per-tile maxima (split-fp16 dgrad)."""
    ci_, co_ = (layer.cout, layer.cin) if dgrad else (layer.cin, layer.cout)
    np_ = split_pieces(layer.H, ci_, co_, dgrad, scaled)
    out = _empty(_pack_numel(layer, np_, dgrad), like=w)
    if np_:
        d = (N.PackDesc * 1)(N.PackDesc(N.ptr(w), N.ptr(out), layer.cin, layer.cout, layer.kind, int(dgrad)))
        N.call("ebsdvae_pack_conv_weights_split", ctypes.addressof(d), 1, np_, N.stream())
    else:
        N.call("ebsdvae_pack_conv_weight", N.ptr(w), N.ptr(out), layer.cin, layer.cout,
               layer.kind, int(dgrad), N.stream())
    return PackedW(out, np_)


class PackSet:
    """Packed forward / input-gradient weights of every conv layer of a plan, refreshed by
    one batched launch per precision (ebsdvae_pack_conv_weights[_split]) per step.  The
    parameter tensors must keep their storage (e.g. views into the trainer's flat buffer)."""

    def __init__(self, plan: "Plan", params):
        self.packs = {}
        descs = {}
        for i, L in enumerate(plan.enc):
            self._add(L, params[L.name + ".weight"], dgrad=i > 0, descs=descs)
        for L in plan.dec:   # every gy comes with per-tile maxima (in_backward[_final])
            self._add(L, params[L.name + ".weight"], dgrad=True, descs=descs)
        self.batches = []
        for np_, lst in sorted(descs.items()):
            if len(lst) > N.MAX_PACK:
                raise RuntimeError(f"PackSet: {len(lst)} packs > {N.MAX_PACK}")
            self.batches.append((np_, (N.PackDesc * len(lst))(*lst), len(lst)))

    def _one(self, L, w, dgrad, descs, scaled=True):
        ci_, co_ = (L.cout, L.cin) if dgrad else (L.cin, L.cout)
        np_ = split_pieces(L.H, ci_, co_, dgrad, scaled)
        t = _empty(_pack_numel(L, np_, dgrad), like=w)
        descs.setdefault(np_, []).append(N.PackDesc(N.ptr(w), N.ptr(t), L.cin, L.cout, L.kind, int(dgrad)))
        return PackedW(t, np_)

    def _add(self, L, w, dgrad, descs, scaled=True):
        # the VALU first conv reads the weight as it is (no pack)
        pf = None if _first_valu(L) else self._one(L, w, False, descs)
        pd = self._one(L, w, True, descs, scaled) if dgrad else None
        self.packs[L.name] = (pf, pd)

    def refresh(self):
        for np_, arr, n in self.batches:
            if np_:
                N.call("ebsdvae_pack_conv_weights_split", ctypes.addressof(arr), n, np_, N.stream())
            else:
                N.call("ebsdvae_pack_conv_weights", ctypes.addressof(arr), n, N.stream())
        return self.packs


def pool_out_ok(layer: ConvLayer, wp) -> bool:
    """The layer's split conv can also emit its max-pooled raw output (FP_POOLOUT).
    EBSDVAE_POOL_OUT=0 turns the pooled hand-off off (A/B timing)."""
    if os.environ.get("EBSDVAE_POOL_OUT", "1") == "0":
        return False
    return bool(wp is not None and wp.pieces and N.call(
        "ebsdvae_conv3x3_split_pool_ok", layer.H, layer.H, layer.cin, layer.cout, wp.pieces))


# The first conv (cin = 1) runs on the VALU with a fixed fma chain (ebsdvae_conv_first_fwd), so
# the first block's backward can recompute y0 from x bit-identically instead of re-reading it
# (ebsdvae_in_bwd_first_apply_wgrad_rc).  EBSDVAE_FIRST_VALU=0: the fp32-MFMA conv + re-read.
_FIRST_VALU = os.environ.get("EBSDVAE_FIRST_VALU", "1") != "0"
# inference skips the full-resolution output of pooled producers (ypool only);
# EBSDVAE_EVAL_Y=1 writes it anyway, for A/B timing
_EVAL_Y = os.environ.get("EBSDVAE_EVAL_Y", "0") == "1"


def _first_valu(layer: ConvLayer) -> bool:
    return (layer.cin == 1 and layer.cout == 32 and layer.src_mode == ACT_RAW and _FIRST_VALU
            and N.call("ebsdvae_conv_first_stat_tiles", layer.H, layer.H) > 0)


# statistics-only first conv (inference): from x's shifted moments in double
# (ebsdvae_conv_first_stats) instead of the fma-chain kernel with its y0 store skipped;
# EBSDVAE_FIRST_GRAM=0 keeps the latter (A/B; bit-identical statistics to training's)
_FIRST_GRAM = os.environ.get("EBSDVAE_FIRST_GRAM", "1") != "0"


def _conv_first(x, layer: ConvLayer, w, b, B, write_y=True):
    """write_y=False: the InstanceNorm statistics only (y None) -- the next conv recomputes y
    from x (conv_forward_first)."""
    H = layer.H
    if not write_y and _FIRST_GRAM and H % 32 == 0 and 256 % H == 0:
        st = _empty(B, layer.cout, 2, like=w)
        _launch("conv3x3_fwd", conv_flops(B, H, H, 1, layer.cout), N.call, "ebsdvae_conv_first_stats",
                N.ptr(x), N.ptr(w), N.ptr(b), N.ptr(st), B, H, H, layer.cout, N.stream(),
                tag=f"fwd  {layer.name:13s} {layer.cin:3d}->{layer.cout:3d} @{H:3d} m0 stats",
                nbytes=4 * x.numel())
        return None, st
    T = N.call("ebsdvae_conv_first_stat_tiles", H, H)
    y = _empty(B, H, H, layer.cout, like=w) if write_y else None
    part = _empty(B, T, layer.cout, 2, like=w)
    st = _empty(B, layer.cout, 2, like=w)
    tag = f"fwd  {layer.name:13s} {layer.cin:3d}->{layer.cout:3d} @{H:3d} m{layer.src_mode} valu"
    _launch("conv3x3_fwd", conv_flops(B, H, H, 1, layer.cout), N.call, "ebsdvae_conv_first_fwd",
            N.ptr(x), N.ptr(w), N.ptr(b), N.ptr(y), N.ptr(part), B, H, H, layer.cout, N.stream(),
            tag=tag + ("" if write_y else " stats"),
            nbytes=4 * (x.numel() + (B * H * H * layer.cout if write_y else 0)))
    N.call("ebsdvae_in_stats_finalize", N.ptr(part), N.ptr(st), B, layer.cout, T, (H * H) // T,
           N.stream())
    if y is not None:
        y.ev_first_valu = True   # in_backward_first may recompute it from x
    return y, st


# The second block's forward recomputes the first block's activation from x while it stages its
# halo (ebsdvae_conv3x3_fwd_split_first): y0 is never read by the forward, and inference never
# writes it (the first conv runs statistics-only).  Bit-identical to reading y0.  Measured
# (round 6): the staging's extra 36 FMAs per item cost the conv more than
# the y0 reads it saves (encoder.1 fwd 336 -> 355 us at B = 256), so it pays only where the
# first conv's 2 GB y0 write goes away too -- inference (c4).  Training keeps y0 (its backward
# reads it) and the two-launch form.
# EBSDVAE_FIRST_FUSE: "eval" (default) inference only, "1" also training, "0" never (A/B).
_FIRST_FUSE = os.environ.get("EBSDVAE_FIRST_FUSE", "eval")
if _FIRST_FUSE not in ("0", "1", "eval"):
    raise ValueError("EBSDVAE_FIRST_FUSE must be 0, 1 or eval")


def first_fuse_ok(plan: Plan, wp1) -> bool:
    """encoder.1 can take its input as x + the first conv (split-fp16 pack, 32 channels)."""
    if not (_FIRST_FUSE != "0" and len(plan.enc) > 1 and _first_valu(plan.enc[0])):
        return False
    L = plan.enc[1]
    return bool(wp1 is not None and wp1.pieces == PIECES_F16 and L.src_mode == ACT_NORM and N.call(
        "ebsdvae_conv3x3_fwd_split_first_ok", L.H, L.H, L.cin, L.cout, wp1.pieces))


def conv_forward_first(x, st0, w0, b0, layer: ConvLayer, w, b, B, wp, pool_out, keep_y=True):
    """conv_forward of the second block with its source lrelu(IN(conv(x, w0) + b0)) recomputed
    from x (st0: the first block's statistics).  Returns (y, st) or (y, st, ypool) as
    conv_forward."""
    H = layer.H
    y = _empty(B, H, H, layer.cout, like=w) if keep_y or not pool_out else None
    T = N.call("ebsdvae_conv3x3_split_stat_tiles", H, H, layer.cout)
    part = _empty(B, T, layer.cout, 2, like=w)
    st = _empty(B, layer.cout, 2, like=w)
    ypool = _empty(B, H // 2, H // 2, layer.cout, like=w) if pool_out else None
    ny = B * H * H * layer.cout
    nb = 4 * (x.numel() + (ny if y is not None else 0) + (ny // 4 if pool_out else 0))
    tag = f"fwd  {layer.name:13s} {layer.cin:3d}->{layer.cout:3d} @{H:3d} m{layer.src_mode} x"
    _launch("conv3x3_fwd", conv_flops(B, H, H, layer.cin, layer.cout), N.call,
            "ebsdvae_conv3x3_fwd_split_first", N.ptr(x), N.ptr(st0), N.ptr(w0), N.ptr(b0),
            N.ptr(wp.t), N.ptr(b), N.ptr(y), N.ptr(ypool), N.ptr(part), N.ptr(st), B, H, H,
            layer.cin, layer.cout, wp.pieces, N.stream(),
            tag=tag + (" pool" if pool_out else ""), pieces=wp.pieces, nbytes=nb)
    if pool_out:
        return y, st, ypool
    return y, st


def conv_forward(src, src_stats, layer: ConvLayer, w, b, B, keep_act=False, wp=None, mode=None,
                 pool_out=False, keep_y=True):
    """One conv block forward: y (B,H,H,cout) pre-norm + IN stats {mean,rstd} (B,cout,2).
    keep_act: also return the conv's logical input (materialised by the kernel), used by
    max-pool-fed layers so their wgrad reads the pooled tensor.  wp: pre-packed weight.
    mode: source mode override (a max-pool-fed layer reading its producer's pooled output
    in ACT_NORM mode).  pool_out: also return ypool = 2x2 max of y (B,H/2,H/2,cout), the
    producer side of that (ebsdvae_conv3x3_fwd_split_pooled); keep_y=False with pool_out
    (inference) writes ypool only and returns y None."""
    H = layer.H
    src_mode = layer.src_mode if mode is None else mode
    if src_mode == ACT_RAW and not keep_act and not pool_out and _first_valu(layer):
        return _conv_first(src, layer, w, b, B)
    if wp is None:
        wp = pack_weight(w, layer, dgrad=False)
    y = _empty(B, H, H, layer.cout, like=w) if keep_y or not pool_out else None
    T = N.call("ebsdvae_conv3x3_split_stat_tiles" if wp.pieces else "ebsdvae_conv3x3_stat_tiles",
               H, H, layer.cout)
    part = _empty(B, T, layer.cout, 2, like=w)
    act = _empty(B, H, H, layer.cin, like=w) if keep_act else None
    tag = f"fwd  {layer.name:13s} {layer.cin:3d}->{layer.cout:3d} @{H:3d} m{layer.src_mode}"
    args = (N.ptr(src), N.ptr(src_stats), src_mode, N.ptr(wp.t), N.ptr(b), N.ptr(y),
            N.ptr(part), N.ptr(act), B, H, H, layer.cin, layer.cout)
    flops = conv_flops(B, H, H, layer.cin, layer.cout)
    ny = B * H * H * layer.cout
    nb = 4 * (src.numel() + (ny if y is not None else 0) + (ny // 4 if pool_out else 0))   # algorithmic I/O
    ypool = None
    st = _empty(B, layer.cout, 2, like=w)
    if pool_out:
        ypool = _empty(B, H // 2, H // 2, layer.cout, like=w)
    if wp.pieces and not keep_act:
        # conv + InstanceNorm statistics finalize (in-kernel where the blocks own whole images)
        _launch("conv3x3_fwd", flops, N.call, "ebsdvae_conv3x3_fwd_split_st", N.ptr(src),
                N.ptr(src_stats), src_mode, N.ptr(wp.t), N.ptr(b), N.ptr(y), N.ptr(ypool),
                N.ptr(part), N.ptr(st), B, H, H, layer.cin, layer.cout, wp.pieces, N.stream(),
                tag=tag + (" pool" if pool_out else ""), pieces=wp.pieces, nbytes=nb)
    else:
        if pool_out:
            raise ValueError("conv_forward: pool_out needs a split pack and no keep_act")
        if wp.pieces:
            _launch("conv3x3_fwd", flops, N.call, "ebsdvae_conv3x3_fwd_split", *args, wp.pieces,
                    N.stream(), tag=tag, pieces=wp.pieces, nbytes=nb)
        else:
            _launch("conv3x3_fwd", flops, N.call, "ebsdvae_conv3x3_fwd", *args, N.stream(), tag=tag,
                    nbytes=nb)
        N.call("ebsdvae_in_stats_finalize", N.ptr(part), N.ptr(st), B, layer.cout, T, (H * H) // T,
               N.stream())
    if pool_out:
        return y, st, ypool
    if keep_act:
        return y, st, act
    return y, st


def in_backward(gnext, pmode, y, st, part=None):
    """gy = d loss / d y through [pool|up] . lrelu . InstanceNorm of one block.
    part: the reduce-pass sums already produced by the fused input-gradient conv that
    computed gnext (conv_dgrad(..., prev=...)), which then holds h = g * lrelu'(xhat), not g
    (csrc/conv_common.h); None: gnext is g and the reduce pass runs here."""
    B, H, W, C = y.shape
    s = N.stream()
    hin = part is not None
    if part is None:
        T = N.call("ebsdvae_in_bwd_tiles", H, W, C)
        part = _f64(B, T, C, 2, device=y.device)
        N.call("ebsdvae_in_bwd_reduce", N.ptr(gnext), pmode, N.ptr(y), N.ptr(st), part.data_ptr(),
               B, H, W, C, s)
    bst = getattr(part, "ev_bst", None)   # finalized by the fused input-gradient conv
    if bst is None:
        bst = _empty(B, C, 2, like=y)
        N.call("ebsdvae_in_bwd_finalize", part.data_ptr(), N.ptr(bst), B, C, part.shape[1], H * W, s)
    gy = _empty_like(y)
    if _FWD_PIECES.get(_PRECISION):
        # per-tile max |gy|: the scale of the split-fp16 input-gradient conv that consumes gy
        Tg = N.call("ebsdvae_in_bwd_apply_tiles", B, H, W, C)
        gmax = _empty(B, Tg, like=y)
        N.call("ebsdvae_in_bwd_happly" if hin else "ebsdvae_in_bwd_apply_max", N.ptr(gnext), pmode,
               N.ptr(y), N.ptr(st), N.ptr(bst), N.ptr(gy), N.ptr(gmax), B, H, W, C, s)
        gy.ev_gmax = gmax
    elif hin:
        N.call("ebsdvae_in_bwd_happly", N.ptr(gnext), pmode, N.ptr(y), N.ptr(st), N.ptr(bst),
               N.ptr(gy), None, B, H, W, C, s)
    else:
        N.call("ebsdvae_in_bwd_apply", N.ptr(gnext), pmode, N.ptr(y), N.ptr(st), N.ptr(bst),
               N.ptr(gy), B, H, W, C, s)
    return gy


def _in_bwd_stats(B, C, T, HW, part, like):
    bst = getattr(part, "ev_bst", None)   # finalized by the fused input-gradient conv
    if bst is not None:
        return bst
    bst = _empty(B, C, 2, like=like)
    N.call("ebsdvae_in_bwd_finalize", part.data_ptr(), N.ptr(bst), B, C, T, HW, N.stream())
    return bst


# ----------------------------------------------------------------------------- side stream
# Weight gradients are off the backward's critical path (in_backward -> input gradient -> ...):
# they run on a second HIP stream, so they overlap the memory-bound InstanceNorm-backward passes
# and the other kernels' tails.  The side stream waits for the main stream before each weight
# gradient (its inputs are ready), and the batched slice reductions run on the side stream too,
# behind the weight gradients they sum.  The main stream waits for the side stream once, at
# the next join: at the end of a batched_wgrad_reduce() block, or -- inside
# deferred_side_join() (the trainer's backward) -- only when that block exits.
# Buffers the side stream touches are kept alive on the host until that join (no
# record_stream: its event records on every free cost the GPU idle time at each join).
# EBSDVAE_WGRAD_STREAM=0 keeps everything on the current stream.
_WG_STREAM = os.environ.get("EBSDVAE_WGRAD_STREAM", "1") != "0"
# Inside a hipGraph capture the side stream forks from and joins back into the capturing
# stream (event edges in the graph).  EBSDVAE_GRAPH_SIDE=0 captures on one stream instead.
_GRAPH_SIDE = os.environ.get("EBSDVAE_GRAPH_SIDE", "1") != "0"
_SIDE = {}
_KEEP = {}    # device -> buffers the side stream uses, released at the join (None: not in use)
_DEFER = 0    # > 0 inside deferred_side_join()


_SERIAL = 0   # > 0 inside serial_streams()


@contextlib.contextmanager
def serial_streams():
    """Keep the weight gradients on the current stream (no overlap), e.g. while per-launch
    durations are being measured: overlapped launches would each be timed with the other's
    work inside (bench.py's probed steps)."""
    global _SERIAL
    _SERIAL += 1
    try:
        yield
    finally:
        _SERIAL -= 1


def _dev_key(device):
    return device.index if device.index is not None else torch.cuda.current_device()


# EBSDVAE_CU_SPLIT=k (experiment): the weight-gradient side stream runs on
# k compute units (CU-mask bits [N - k, N), N / 8 of them on every XCD) and cu_split_main()
# gives the complementary N - k for the input-gradient chain, whose persistent conv kernels then
# launch N - k blocks (ebsdvae_stream_create_cus).  The caller runs the step on that stream.
_CU_SPLIT = int(os.environ.get("EBSDVAE_CU_SPLIT", "0"))
_CU_MAIN = {}


def _cu_stream(device, first, count):
    import ctypes as C
    out = C.c_void_p()
    with torch.cuda.device(device):
        N.call("ebsdvae_stream_create_cus", first, count, C.byref(out))
    return torch.cuda.ExternalStream(out.value, device=device)


def cu_split_main(device):
    """The CU-partitioned main stream of `device` under EBSDVAE_CU_SPLIT (None otherwise)."""
    if _CU_SPLIT <= 0:
        return None
    key = _dev_key(device)
    if key not in _CU_MAIN:
        ncu = torch.cuda.get_device_properties(key).multi_processor_count
        _CU_MAIN[key] = _cu_stream(torch.device("cuda", key), 0, ncu - _CU_SPLIT)
    return _CU_MAIN[key]


def side_stream(device):
    """The weight-gradient side stream of `device` (created on first use; CU-masked to
    EBSDVAE_CU_SPLIT compute units when set)."""
    key = _dev_key(device)
    if key not in _SIDE:
        if _CU_SPLIT > 0:
            ncu = torch.cuda.get_device_properties(key).multi_processor_count
            _SIDE[key] = _cu_stream(torch.device("cuda", key), ncu - _CU_SPLIT, _CU_SPLIT)
        else:
            _SIDE[key] = torch.cuda.Stream(device=device)
    return _SIDE[key]


def side_streams_enabled() -> bool:
    """Work may go to the side stream now (not disabled, not inside serial_streams(), and not
    a capture that keeps everything on one stream)."""
    if not _WG_STREAM or _SERIAL:
        return False
    return _GRAPH_SIDE or not torch.cuda.is_current_stream_capturing()


def _side_stream(device):
    if not _WG_STREAM or _SERIAL:
        return None
    if not _GRAPH_SIDE and torch.cuda.is_current_stream_capturing():
        return None
    return side_stream(device)


# EBSDVAE_LIGHT_EVENTS=0: fork / join through torch's Stream.wait_stream (system-scope fence)
_LIGHT_EVENTS = os.environ.get("EBSDVAE_LIGHT_EVENTS", "1") != "0"


def stream_wait(waiter, signaler):
    """`waiter` (a torch Stream) waits for the work enqueued on `signaler` so far."""
    if _LIGHT_EVENTS:
        N.call("ebsdvae_stream_wait", waiter.cuda_stream, signaler.cuda_stream)
    else:
        waiter.wait_stream(signaler)


# EBSDVAE_KFORK=0: every fork records an event on the main stream (A/B).  Otherwise the
# backward arms a kernel-attached fork before each InstanceNorm-backward apply whose gy a
# weight gradient takes: the apply launch itself signals the event (ebsdvae_fork_arm /
# ebsdvae_fork_wait), so no record packet sits between the apply and the input-gradient conv.
_KFORK = os.environ.get("EBSDVAE_KFORK", "1") != "0"


def fork_arm(device) -> bool:
    """Arm a kernel-attached fork for the next InstanceNorm-backward apply on the current
    stream.  Returns the token to pass to the weight gradient that consumes that apply's gy
    (conv_wgrad(..., fork=...)); False (nothing armed) when the weight gradients will not go
    to the side stream.  The armed state lives in the library per host thread: a later arm
    replaces it, and only a conv_wgrad holding the token waits on it."""
    if _KFORK and _LIGHT_EVENTS and _side_stream(device) is not None \
            and not torch.cuda.is_current_stream_capturing():
        N.call("ebsdvae_fork_arm", N.stream())
        return True
    return False


def _side_use(device, *tensors, fork=False):
    """Fork the side stream from the current stream and keep `tensors` alive until the join.
    fork: fork_arm()'s token -- the side stream waits for the armed apply launch only (the
    last main-stream work the caller's inputs depend on) instead of an event recorded now."""
    key = _dev_key(device)
    side = side_stream(device)
    cur = torch.cuda.current_stream(device)
    if fork:
        N.call("ebsdvae_fork_wait", side.cuda_stream, cur.cuda_stream)
    else:
        stream_wait(side, cur)
    keep = _KEEP.get(key)
    if keep is None:
        keep = _KEEP[key] = []
    keep.extend(t for t in tensors if t is not None)
    return side


def _side_pending(device) -> bool:
    return _KEEP.get(_dev_key(device)) is not None


def _join_side(device):
    """The current stream waits for the side stream's work so far; the buffers it used are
    released (any later use of them is ordered behind this wait)."""
    key = _dev_key(device)
    if _KEEP.get(key) is not None:   # only a side stream that took work since the last join
        stream_wait(torch.cuda.current_stream(device), _SIDE[key])
        _KEEP[key] = None


@contextlib.contextmanager
def deferred_side_join(device):
    """Batched reductions inside the block leave their results on the side stream; the
    current stream joins it once, when the block exits."""
    global _DEFER
    _DEFER += 1
    try:
        yield
    finally:
        _DEFER -= 1
        _join_side(device)


# EBSDVAE_FINAL_REDUCE_SIDE=1: the encoder's last reduction batch on the side stream as through
# round 6's middle (A/B)
_ON_MAIN_FINAL = os.environ.get("EBSDVAE_FINAL_REDUCE_SIDE", "0") in ("", "0")
# Weight-gradient slice reductions queued inside `batched_wgrad_reduce()` run as ONE batched
# pair of launches when the block exits (ebsdvae_wgrad_reduce_batch) instead of two launches
# per layer; outside such a block they run immediately.  Results are bit-identical.
_RQ = None


@contextlib.contextmanager
def batched_wgrad_reduce(on_main: bool = False):
    """on_main: the batch is the step's last work (the encoder backward): it runs on the current
    stream after one join of the side stream, instead of on the side stream behind a fork of the
    current one and joined again (two cross-stream hops, ≈13 µs each at the end of the step)."""
    global _RQ
    outer, q = _RQ, []
    _RQ = q
    try:
        yield
    finally:
        _RQ = outer
        _flush_reduces(q, on_main=on_main)


def _flush_reduces(q, on_main: bool = False):
    if not q:
        return
    dev = q[0][0].device
    if on_main and _ON_MAIN_FINAL and _side_pending(dev):
        _join_side(dev)   # the weight gradients' partials are complete once the side stream is
    side = side_stream(dev) if _side_pending(dev) else None
    if side is not None:
        # behind the weight gradients on the side stream; partials made on the current
        # stream (the fused network-end passes) are ordered by a fork -- only then, so a
        # batch of side-stream partials does not wait for the current stream
        mine = [t for e in q if not e[8] for t in e[:2]]
        if mine:
            _side_use(dev, *mine)
        ctx = torch.cuda.stream(side)
    else:
        ctx = contextlib.nullcontext()
    with ctx:
        for i in range(0, len(q), N.MAX_WGRAD_BATCH):
            chunk = q[i:i + N.MAX_WGRAD_BATCH]
            descs = (N.WgradReduceDesc * len(chunk))(*[
                N.WgradReduceDesc(N.ptr(wp), N.ptr(bp), N.ptr(dw), N.ptr(db), S_, cin, cout, kind)
                for wp, bp, S_, cin, cout, kind, dw, db, _ in chunk])
            nbytes = N.call("ebsdvae_wgrad_reduce_batch_work", ctypes.addressof(descs), len(chunk))
            work = _f64(nbytes // 8, device=dev)
            N.call("ebsdvae_wgrad_reduce_batch", ctypes.addressof(descs), len(chunk),
                   work.data_ptr(), N.stream())
            if side is not None:
                _KEEP[_dev_key(dev)].append(work)
    if side is not None and not _DEFER:
        _join_side(dev)


def _reduce_slices(wpart, bpart, S_, cin, cout, kind, dw, db, on_side=False):
    """on_side: the partials were written on the side stream (conv_wgrad)."""
    e = (wpart, bpart, S_, cin, cout, kind, dw, db, on_side)
    if _RQ is not None:
        _RQ.append(e)
    elif _side_pending(wpart.device):
        _flush_reduces([e])   # on the side stream, then joined
    else:
        nbytes = N.call("ebsdvae_wgrad_reduce_work", S_, cin, cout)
        work = _f64(nbytes // 8, device=wpart.device)
        N.call("ebsdvae_wgrad_reduce", N.ptr(wpart), N.ptr(bpart), S_, N.ptr(dw), N.ptr(db), cin,
               cout, kind, work.data_ptr(), N.stream())


def in_backward_final(g1, w14, y, st, dw14, db14):
    """Backward of the last conv block + the final conv(32->1) (latice/model.py:147-148):
    returns gy of the last block and writes the final conv's dW/db."""
    B, H, W, C = y.shape
    T = N.call("ebsdvae_in_bwd_tiles", H, W, C)
    S_ = B * T
    part = _f64(B, T, C, 2, device=y.device)
    wpart = _empty(S_, 9, 1, C, like=y)
    bpart = _empty(S_, 1, like=y)
    N.call("ebsdvae_in_bwd_final_reduce", N.ptr(g1), N.ptr(w14), N.ptr(y), N.ptr(st),
           part.data_ptr(), N.ptr(wpart), N.ptr(bpart), B, H, W, C, N.stream())
    bst = _in_bwd_stats(B, C, T, H * W, part, y)
    gy = _empty_like(y)
    if _FWD_PIECES.get(_PRECISION):
        # per-tile max |gy|: the scale of the split-fp16 convs that consume gy
        gmax = _empty(B, N.call("ebsdvae_in_bwd_final_tiles", H, W), like=y)
        N.call("ebsdvae_in_bwd_final_apply_max", N.ptr(g1), N.ptr(w14), N.ptr(y), N.ptr(st),
               N.ptr(bst), N.ptr(gy), N.ptr(gmax), B, H, W, C, N.stream())
        gy.ev_gmax = gmax
    else:
        N.call("ebsdvae_in_bwd_final_apply", N.ptr(g1), N.ptr(w14), N.ptr(y), N.ptr(st), N.ptr(bst),
               N.ptr(gy), B, H, W, C, N.stream())
    _reduce_slices(wpart, bpart, S_, C, 1, KIND_CONV, dw14, db14)
    return gy


# ----------------------------------------------------------------------------- network end
# ebsdvae_net_end: the final conv's forward, the BCE part of the loss and its logit gradient, and
# the last block's InstanceNorm-backward reduce + the final conv's gradient slices in one pass
# over y13 (the training step; EBSDVAE_NET_END=0 keeps the separate kernels for A/B timing).
_NET_END = os.environ.get("EBSDVAE_NET_END", "1") != "0"
# its contractions on the split-fp16 MFMA (round 6); EBSDVAE_NET_END_MFMA=0: the VALU form (A/B)
_NET_END_MFMA = os.environ.get("EBSDVAE_NET_END_MFMA", "1") != "0"


@dataclass
class NetEnd:
    g1: torch.Tensor      # (B, S, S) logit gradient of the mean BCE
    part: torch.Tensor    # (B, T, C, 2) float64 reduce sums of the last block
    wpart: torch.Tensor   # (B*T, 9, 1, C) final-conv weight-gradient slices
    bpart: torch.Tensor   # (B*T,)
    bce: torch.Tensor     # (B, T) per-band BCE sums
    tiles: int


def net_end_ok(plan: Plan) -> bool:
    S = plan.image_size
    return _NET_END and plan.inplanes == 32 and N.call("ebsdvae_net_end_tiles", S, S) > 0


def network_end(plan: Plan, saved, params, x, g_loss=None, scale: float = 1.0):
    """x_hat and a NetEnd from the decoder's saved last block (decoder_forward(final=False))."""
    y13, st13 = saved[plan.dec[-1].name]
    B, H, W, C = y13.shape
    T = N.call("ebsdvae_net_end_tiles", H, W)
    x_hat = _empty(B, 1, H, W, like=y13)
    g1 = _empty(B, H, W, like=y13)
    bce = _empty(B, T, like=y13)
    part = _f64(B, T, C, 2, device=y13.device)
    wpart = _empty(B * T, 9, 1, C, like=y13)
    bpart = _empty(B * T, like=y13)
    N.call("ebsdvae_net_end" if _NET_END_MFMA else "ebsdvae_net_end_valu", N.ptr(y13), N.ptr(st13), N.ptr(params["decoder.14.weight"]),
           N.ptr(params["decoder.14.bias"]), N.ptr(x), N.ptr(g_loss), float(scale), N.ptr(x_hat),
           N.ptr(g1), N.ptr(bce), part.data_ptr(), N.ptr(wpart), N.ptr(bpart), B, H, W, C,
           N.stream())
    return x_hat, NetEnd(g1, part, wpart, bpart, bce, T)


def in_backward_final_from(end: NetEnd, w14, y, st, dw14, db14):
    """in_backward_final with the reduce pass already done by network_end."""
    B, H, W, C = y.shape
    bst = _in_bwd_stats(B, C, end.tiles, H * W, end.part, y)
    gy = _empty_like(y)
    if _FWD_PIECES.get(_PRECISION):
        gmax = _empty(B, N.call("ebsdvae_in_bwd_final_tiles", H, W), like=y)
        N.call("ebsdvae_in_bwd_final_apply_max", N.ptr(end.g1), N.ptr(w14), N.ptr(y), N.ptr(st),
               N.ptr(bst), N.ptr(gy), N.ptr(gmax), B, H, W, C, N.stream())
        gy.ev_gmax = gmax
    else:
        N.call("ebsdvae_in_bwd_final_apply", N.ptr(end.g1), N.ptr(w14), N.ptr(y), N.ptr(st), N.ptr(bst),
               N.ptr(gy), B, H, W, C, N.stream())
    _reduce_slices(end.wpart, end.bpart, B * end.tiles, C, 1, KIND_CONV, dw14, db14)
    return gy


def in_backward_first(gnext, y, st, x, dw0, db0, part=None, w0=None, b0=None):
    """Backward of the first conv block (latice/model.py:110): writes dW/db of the 1->32
    conv directly from the InstanceNorm-backward apply pass (gy is never materialised).
    part: reduce-pass sums from the fused input-gradient conv (None: reduce here).
    w0, b0: the first conv's parameters; with them, and y from ebsdvae_conv_first_fwd, y is
    recomputed from x instead of read."""
    B, H, W, C = y.shape
    hin = part is not None   # gnext is a fused input gradient's h (see in_backward)
    if part is None:
        T = N.call("ebsdvae_in_bwd_tiles", H, W, C)
        part = _f64(B, T, C, 2, device=y.device)
        N.call("ebsdvae_in_bwd_reduce", N.ptr(gnext), P_ID, N.ptr(y), N.ptr(st), part.data_ptr(),
               B, H, W, C, N.stream())
    bst = _in_bwd_stats(B, C, part.shape[1], H * W, part, y)
    T = N.call("ebsdvae_in_bwd_tiles", H, W, C)
    S_ = B * T
    wpart = _empty(S_, 9, C, 1, like=y)
    bpart = _empty(S_, C, like=y)
    if w0 is not None and getattr(y, "ev_first_valu", False):
        N.call("ebsdvae_in_bwd_first_happly_wgrad_rc" if hin else "ebsdvae_in_bwd_first_apply_wgrad_rc",
               N.ptr(gnext), N.ptr(w0), N.ptr(b0), N.ptr(st), N.ptr(bst), N.ptr(x), N.ptr(wpart),
               N.ptr(bpart), B, H, W, C, N.stream())
    else:
        N.call("ebsdvae_in_bwd_first_happly_wgrad" if hin else "ebsdvae_in_bwd_first_apply_wgrad",
               N.ptr(gnext), N.ptr(y), N.ptr(st), N.ptr(bst), N.ptr(x), N.ptr(wpart), N.ptr(bpart),
               B, H, W, C, N.stream())
    _reduce_slices(wpart, bpart, S_, 1, C, KIND_CONV, dw0, db0)


def conv_wgrad(src, src_stats, src_mode, gy, cin, cout, kind, dw, db, normalized=None,
               fork=False):
    """normalized: src is a normalised activation (default: the NORM modes); the split-fp16
    weight gradient (f16x3, gy with per-tile maxima) scales only gy, so it needs one.
    Runs on the side stream (see _side_stream); dw/db are written by the slice reduction on
    the caller's stream."""
    side = _side_stream(gy.device)
    if side is None:
        return _conv_wgrad(src, src_stats, src_mode, gy, cin, cout, kind, dw, db, normalized)
    side = _side_use(gy.device, src, src_stats, gy, getattr(gy, "ev_gmax", None), fork=fork)
    with torch.cuda.stream(side):
        wpart, bpart, S_ = _conv_wgrad(src, src_stats, src_mode, gy, cin, cout, kind, dw, db,
                                       normalized, reduce=False)
    _KEEP[_dev_key(gy.device)].extend((wpart, bpart))
    _reduce_slices(wpart, bpart, S_, cin, cout, kind, dw, db, on_side=True)


def _conv_wgrad(src, src_stats, src_mode, gy, cin, cout, kind, dw, db, normalized=None,
                reduce=True):
    B, H, W, _ = gy.shape if gy.dim() == 4 else (*gy.shape, 1)
    if normalized is None:
        normalized = src_mode in (ACT_NORM, ACT_NORM_UP)
    gmax = getattr(gy, "ev_gmax", None)
    nbw = 4 * (src.numel() + gy.numel())   # algorithmic I/O: source activation + gradient
    if (gmax is not None and normalized and _FWD_PIECES.get(_PRECISION)
            and os.environ.get("EBSDVAE_WGRAD_F16", "1") != "0"):
        S_ = N.call("ebsdvae_conv3x3_wgrad_split_slices", B, H, W, cin, cout, PIECES_F16)
        if S_ > 0:
            wpart = _empty(S_, 9, cout, cin, like=gy)
            bpart = _empty(S_, cout, like=gy)
            _launch("conv3x3_wgrad", conv_flops(B, H, W, cin, cout), N.call,
                    "ebsdvae_conv3x3_wgrad_f16", N.ptr(src), N.ptr(src_stats), src_mode, N.ptr(gy),
                    N.ptr(gmax), gmax.shape[1], N.ptr(wpart), N.ptr(bpart), B, H, W, cin, cout,
                    N.stream(), tag=f"wgrad {cin:3d}->{cout:3d} @{H:3d} m{src_mode} f16",
                    pieces=PIECES_F16, nbytes=nbw)
            if not reduce:
                return wpart, bpart, S_
            _reduce_slices(wpart, bpart, S_, cin, cout, kind, dw, db)
            return
    np_ = _PIECES[_PRECISION]
    S_ = N.call("ebsdvae_conv3x3_wgrad_split_slices", B, H, W, cin, cout, np_) if np_ else -1
    if S_ <= 0:
        np_ = 0
        S_ = N.call("ebsdvae_conv3x3_wgrad_slices", B, H, W, cin, cout)
    if S_ <= 0:
        raise RuntimeError(f"wgrad: unsupported shape {H}x{W}")
    wpart = _empty(S_, 9, cout, cin, like=gy)
    bpart = _empty(S_, cout, like=gy)
    s = N.stream()
    args = (N.ptr(src), N.ptr(src_stats), src_mode, N.ptr(gy), N.ptr(wpart), N.ptr(bpart), B, H, W,
            cin, cout)
    tag = f"wgrad {cin:3d}->{cout:3d} @{H:3d} m{src_mode}"
    if np_:
        _launch("conv3x3_wgrad", conv_flops(B, H, W, cin, cout), N.call, "ebsdvae_conv3x3_wgrad_split",
                *args, np_, s, tag=tag, pieces=np_, nbytes=nbw)
    else:
        _launch("conv3x3_wgrad", conv_flops(B, H, W, cin, cout), N.call, "ebsdvae_conv3x3_wgrad",
                *args, s, tag=tag, nbytes=nbw)
    if not reduce:
        return wpart, bpart, S_
    _reduce_slices(wpart, bpart, S_, cin, cout, kind, dw, db)


def conv_dgrad(gy, layer: ConvLayer, w, prev=None, wd=None, sum_up=False, ypool=None):
    """Input gradient of `layer`.  prev = (y_prev, st_prev, pmode_prev) of the block feeding
    it: the previous block's InstanceNorm-backward reduce is then fused into the epilogue and
    (gin, part) is returned for in_backward(..., part=part); gin is then h = g * lrelu'(xhat),
    not g (csrc/conv_common.h).
    sum_up (pmode_prev == P_UP): where the split kernel supports it, gin is returned already
    2x2-summed, i.e. at the previous block's resolution (then in_backward takes it as P_ID).
    ypool (pmode_prev == P_POOL): the previous block's max-pooled raw output, which its forward
    conv emitted (FP_POOLOUT).  Only the window maximum receives gradient, and the pool adjoint
    leaves the reduce sums  sum g*lrelu'(xhat), sum g*lrelu'(xhat)*xhat  unchanged when xhat is
    taken at the maximum: xhat(max y) = (ypool - mean) * rstd, as IN's scale is positive.  So the
    reduce reads ypool in identity mode -- a quarter of the bytes of the 2x2 windows of y_prev
    and no argmax -- while the apply (in_backward) still routes through y_prev's windows."""
    B, H, W, _ = gy.shape
    hw_prev = None if prev is None else prev[0].shape[1] * prev[0].shape[2]
    if prev is not None and prev[2] == P_POOL and ypool is not None and \
            os.environ.get("EBSDVAE_POOL_REDUCE", "1") != "0":
        prev = (ypool, prev[1], P_ID)
    if wd is None:
        wd = pack_weight(w, layer, dgrad=True, scaled=getattr(gy, "ev_gmax", None) is not None)
    if (sum_up and prev is not None and prev[2] == P_UP and wd.pieces
            and os.environ.get("EBSDVAE_UPSUM", "1") != "0"
            and N.call("ebsdvae_conv3x3_split_pool_ok", H, W, layer.cout, layer.cin, wd.pieces)):
        prev = (prev[0], prev[1], P_UPSUM)
    if prev is not None and prev[2] == P_UPSUM:
        gin = _empty(B, H // 2, W // 2, layer.cin, like=gy)
    else:
        gin = _empty(B, H, W, layer.cin, like=gy)
    tag = f"dgrad {layer.name:13s} {layer.cout:3d}->{layer.cin:3d} @{H:3d}"
    flops = conv_flops(B, H, W, layer.cin, layer.cout)
    nbd = 4 * (gy.numel() + gin.numel())   # algorithmic I/O: output gradient in, input gradient out
    if wd.pieces == PIECES_F16:
        gmax = getattr(gy, "ev_gmax", None)
        if gmax is None:
            raise RuntimeError("conv_dgrad: split-fp16 input gradient needs gy's per-tile maxima "
                               "(in_backward under f16x3)")
        if prev is None:
            _launch("conv3x3_fwd", flops, N.call, "ebsdvae_conv3x3_dgrad_inbwd_f16", N.ptr(gy),
                    N.ptr(gmax), gmax.shape[1], N.ptr(wd.t), N.ptr(gin), None, None, -1, None, B, H,
                    W, layer.cout, layer.cin, N.stream(), tag=tag, pieces=wd.pieces, nbytes=nbd)
            return gin
        # fused reduce + finalize of the previous block's InstanceNorm backward: part carries
        # the finalized statistics (part.ev_bst) for in_backward / in_backward_first
        y_prev, st_prev, pmode = prev
        T = N.call("ebsdvae_conv3x3_split_stat_tiles", H, W, layer.cin)
        part = _f64(B, T, layer.cin, 2, device=gy.device)
        bst = _empty(B, layer.cin, 2, like=gy)
        _launch("conv3x3_fwd", flops, N.call, "ebsdvae_conv3x3_dgrad_inbwd_f16_bst", N.ptr(gy),
                N.ptr(gmax), gmax.shape[1], N.ptr(wd.t), N.ptr(gin), N.ptr(y_prev), N.ptr(st_prev),
                pmode, part.data_ptr(), N.ptr(bst), hw_prev, B, H, W,
                layer.cout, layer.cin, N.stream(), tag=tag + " +inbwd", pieces=wd.pieces, nbytes=nbd)
        part.ev_bst = bst
        return gin, part
    if prev is None:
        if wd.pieces:
            _launch("conv3x3_fwd", flops, N.call, "ebsdvae_conv3x3_dgrad_inbwd_split", N.ptr(gy),
                    N.ptr(wd.t), N.ptr(gin), None, None, -1, None, B, H, W, layer.cout, layer.cin,
                    wd.pieces, N.stream(), tag=tag, pieces=wd.pieces, nbytes=nbd)
        else:
            _launch("conv3x3_fwd", flops, N.call, "ebsdvae_conv3x3_fwd", N.ptr(gy), None, ACT_RAW,
                    N.ptr(wd.t), None, N.ptr(gin), None, None, B, H, W, layer.cout, layer.cin,
                    N.stream(), tag=tag, nbytes=nbd)
        return gin
    y_prev, st_prev, pmode = prev
    T = N.call("ebsdvae_conv3x3_split_stat_tiles" if wd.pieces else "ebsdvae_conv3x3_stat_tiles",
               H, W, layer.cin)
    part = _f64(B, T, layer.cin, 2, device=gy.device)
    args = (N.ptr(gy), N.ptr(wd.t), N.ptr(gin), N.ptr(y_prev), N.ptr(st_prev), pmode,
            part.data_ptr(), B, H, W, layer.cout, layer.cin)
    if wd.pieces:
        _launch("conv3x3_fwd", flops, N.call, "ebsdvae_conv3x3_dgrad_inbwd_split", *args, wd.pieces,
                N.stream(), tag=tag + " +inbwd", pieces=wd.pieces, nbytes=nbd)
    else:
        _launch("conv3x3_fwd", flops, N.call, "ebsdvae_conv3x3_dgrad_inbwd", *args, N.stream(),
                tag=tag + " +inbwd", nbytes=nbd)
    return gin, part


# ebsdvae_conv3x3_dwgrad_f16 (csrc/conv_fused.hip): the input gradient (with the previous
# block's fused InstanceNorm-backward reduce) and the weight gradient of a 32 -> 32 layer in one
# pass over gy and y_prev (encoder.1, decoder.13).  Opt-in (EBSDVAE_DWFUSE=1): measured in the
# B = 256 step it is 0.17 ms slower than the separate kernels, whose weight gradient overlaps the
# next input gradient on the side stream.
_DWFUSE = os.environ.get("EBSDVAE_DWFUSE", "0") == "1"


def dwgrad_ok(gy, layer: ConvLayer, wd, src_mode, prev_pmode) -> bool:
    """The fused kernel covers `layer` (split-fp16 gy with maxima, 32 channels, a source that is
    the normalised [upsampled] previous block and the matching reduce routing)."""
    if wd is None or wd.pieces != PIECES_F16 or getattr(gy, "ev_gmax", None) is None:
        return False
    if (src_mode, prev_pmode) not in ((ACT_NORM, P_ID), (ACT_NORM_UP, P_UP)):
        return False
    B, H, W, _ = gy.shape
    return N.call("ebsdvae_conv3x3_dwgrad_slices", B, H, W, layer.cin, layer.cout) > 0


def conv_dwgrad(gy, layer: ConvLayer, wd, src, sst, src_mode, dw, db):
    """Fused input + weight gradient (dwgrad_ok): returns (gin, part) like conv_dgrad(...,
    prev=(src, sst, P_ID | P_UP), sum_up=True) -- gin is h at src's resolution -- and queues the
    weight gradient's slice reduction like conv_wgrad."""
    B, H, W, _ = gy.shape
    gmax = gy.ev_gmax
    S_ = N.call("ebsdvae_conv3x3_dwgrad_slices", B, H, W, layer.cin, layer.cout)
    T = N.call("ebsdvae_conv3x3_dwgrad_stat_tiles", H, W)
    Hs, Ws = src.shape[1], src.shape[2]
    gin = _empty(B, Hs, Ws, layer.cin, like=gy)
    part = _f64(B, T, layer.cin, 2, device=gy.device)
    wpart = _empty(S_, 9, layer.cout, layer.cin, like=gy)
    bpart = _empty(S_, layer.cout, like=gy)
    tag = f"dwgrad {layer.name:13s} {layer.cout:3d}->{layer.cin:3d} @{H:3d} m{src_mode}"
    flops = 2 * conv_flops(B, H, W, layer.cin, layer.cout)
    nb = 4 * (gy.numel() + src.numel() + gin.numel())   # algorithmic I/O: gy, y_prev in, h out
    _launch("conv3x3_dwgrad", flops, N.call, "ebsdvae_conv3x3_dwgrad_f16", N.ptr(gy), N.ptr(gmax),
            gmax.shape[1], N.ptr(wd.t), N.ptr(src), N.ptr(sst), src_mode, N.ptr(gin),
            part.data_ptr(), N.ptr(wpart), N.ptr(bpart), B, H, W, layer.cin, layer.cout, N.stream(),
            tag=tag, pieces=wd.pieces, nbytes=nb)
    _reduce_slices(wpart, bpart, S_, layer.cin, layer.cout, layer.kind, dw, db)
    return gin, part


def _grad_buf(grads, name, like):
    if grads is not None and name in grads:
        return grads[name]
    return _empty_like(like)


# ----------------------------------------------------------------------------- encoder
def _wp(packs, name, k):
    return None if packs is None else packs[name][k]


def encoder_forward(plan: Plan, x, params, packs=None, train=True, packs_ready=None):
    """x: (B,1,S,S) fp32 (== NHWC).  Returns (enc_out NHWC (B,s,s,C), saved).
    packs: PackSet.refresh() result (None: pack each weight on the fly).
    train=False (inference): skip the pooled activations only the weight gradient needs.
    packs_ready: called once before the first layer that reads `packs` (the trainer packs on
    the side stream while the unpacked VALU first conv runs)."""
    B = x.shape[0]
    saved = {}
    src, sst = x, None
    pooled = None   # the previous layer's max-pooled raw output, when it emitted one
    fuse1 = None    # encoder.1 recomputes the first block from x: (w0, b0, st0)
    for i, L in enumerate(plan.enc):
        w, b = params[L.name + ".weight"], params[L.name + ".bias"]
        if packs_ready is not None and not (i == 0 and _first_valu(L)):
            packs_ready()
            packs_ready = None
        wp = _wp(packs, L.name, 0)
        if wp is None and not _first_valu(L):
            wp = pack_weight(w, L, dgrad=False)
        nxt = plan.enc[i + 1] if i + 1 < len(plan.enc) else None
        if i == 0 and _first_valu(L) and len(plan.enc) > 1 and \
                (_FIRST_FUSE == "1" or (_FIRST_FUSE == "eval" and not train)):
            L1 = plan.enc[1]
            wp1 = _wp(packs, L1.name, 0)
            if wp1 is None:
                wp1 = pack_weight(params[L1.name + ".weight"], L1, dgrad=False)
            if first_fuse_ok(plan, wp1):
                # training keeps y0 for the backward (the first block's pass recomputes it, the
                # second conv's weight and input gradients read it); inference never writes it
                y, st = _conv_first(x, L, w, b, B, write_y=train)
                fuse1 = (w, b, st)
                if train:
                    saved[L.name] = (y, st)
                src, sst = y, st
                continue
        # producer of a max-pool-fed layer: emit the pooled raw output in the epilogue, so
        # the consumer (and its wgrad) read (H/2)^2 pixels in ACT_NORM mode instead of
        # pooling the full-resolution output while staging
        pool_out = (nxt is not None and nxt.src_mode == ACT_NORM_POOL and L.src_mode == ACT_NORM
                    and pool_out_ok(L, wp))
        if i == 1 and fuse1 is not None:
            w0, b0, st0 = fuse1
            if pool_out:
                y, st, ypool = conv_forward_first(x, st0, w0, b0, L, w, b, B, wp, True,
                                                  keep_y=train or _EVAL_Y)
            else:
                y, st = conv_forward_first(x, st0, w0, b0, L, w, b, B, wp, False)
        elif pooled is not None:
            y, st = conv_forward(pooled, sst, L, w, b, B, wp=wp, mode=ACT_NORM)
            if train:
                saved[L.name + ".pool_in"] = pooled
        elif train and L.src_mode == ACT_NORM_POOL:
            y, st, act = conv_forward(src, sst, L, w, b, B, keep_act=True, wp=wp)
            saved[L.name + ".act_in"] = act
        elif pool_out:   # inference: only the pooled output is read downstream
            y, st, ypool = conv_forward(src, sst, L, w, b, B, wp=wp, pool_out=True,
                                        keep_y=train or _EVAL_Y)
        else:
            y, st = conv_forward(src, sst, L, w, b, B, wp=wp)
        pooled = ypool if pool_out else None
        if train:
            saved[L.name] = (y, st)
        src, sst = y, st
    _record(plan.enc, saved)
    s, C = plan.enc_side, plan.enc_channels
    out = _empty(B, s, s, C, like=x)
    N.call("ebsdvae_act_apply", N.ptr(src), N.ptr(sst), ACT_NORM_POOL, N.ptr(out), B, s, s, C,
           N.stream())
    return out, saved


def encoder_backward(plan: Plan, g_enc, x, saved, params, grads=None, need_gx=False, packs=None,
                     after_wgrad=None):
    """g_enc: grad of the encoder output (B,s,s,C) NHWC.  Returns (grads dict, gx or None).
    The layers' weight-gradient reductions run batched when it returns.  after_wgrad:
    {layer name: callable}: once that layer's weight gradient is issued, the reductions queued
    so far are flushed (on the stream the weight gradients run on) and the callable runs -- the
    trainer starts the all-reduce of the gradients finished by then (trainer.py)."""
    with batched_wgrad_reduce(on_main=True):
        return _encoder_backward(plan, g_enc, x, saved, params, grads, need_gx, packs,
                                 after_wgrad or {})


def _flush_queued_reduces():
    """Issue the weight-gradient reductions queued in the current batched_wgrad_reduce block."""
    if _RQ:
        q = list(_RQ)
        _RQ.clear()
        _flush_reduces(q)


def _encoder_backward(plan, g_enc, x, saved, params, grads, need_gx, packs, after_wgrad):
    out = {}

    def done(name):
        if name in after_wgrad:
            _flush_queued_reduces()
            after_wgrad[name]()

    g_next, part = g_enc, None
    gx = None
    for i in reversed(range(len(plan.enc))):
        L = plan.enc[i]
        y, st = saved[L.name]
        if i == 0 and not need_gx:
            # first conv's weight gradient fused into its block's InstanceNorm backward
            wn, bn = L.name + ".weight", L.name + ".bias"
            dw = _grad_buf(grads, wn, params[wn])
            db = _grad_buf(grads, bn, params[bn])
            in_backward_first(g_next, y, st, x, dw, db, part=part, w0=params[wn], b0=params[bn])
            out[wn], out[bn] = dw, db
            done(L.name)
            break
        P = plan.enc[i - 1] if i > 0 else None
        fused = (P is not None and L.src_mode == ACT_NORM and L.name + ".pool_in" not in saved
                 and _DWFUSE and _FWD_PIECES.get(_PRECISION) and L.cin == 32 and L.cout == 32)
        fk = False if fused else fork_arm(y.device)   # the weight gradient forks on the apply
        gy = in_backward(g_next, L.pmode, y, st, part=part)
        wn, bn = L.name + ".weight", L.name + ".bias"
        if fused and dwgrad_ok(gy, L, _wp(packs, L.name, 1), ACT_NORM, P.pmode):
            dw = _grad_buf(grads, wn, params[wn])
            db = _grad_buf(grads, bn, params[bn])
            y_p, st_p = saved[P.name]
            g_next, part = conv_dwgrad(gy, L, _wp(packs, L.name, 1), y_p, st_p, ACT_NORM, dw, db)
            out[wn], out[bn] = dw, db
            done(L.name)
            continue
        mode = L.src_mode
        if i == 0:
            src, sst = x, None
        elif L.name + ".pool_in" in saved:   # the producer's pooled raw output
            src, sst, mode = saved[L.name + ".pool_in"], saved[plan.enc[i - 1].name][1], ACT_NORM
        elif L.src_mode == ACT_NORM_POOL:
            src, sst, mode = saved[L.name + ".act_in"], None, ACT_RAW
        else:
            src, sst = saved[plan.enc[i - 1].name]
        dw = _grad_buf(grads, wn, params[wn])
        db = _grad_buf(grads, bn, params[bn])
        # every source but the raw input image is a normalised activation (.act_in included)
        conv_wgrad(src, sst, mode, gy, L.cin, L.cout, L.kind, dw, db, normalized=i > 0, fork=fk)
        out[wn], out[bn] = dw, db
        done(L.name)
        if i > 0:
            P = plan.enc[i - 1]
            g_next, part = conv_dgrad(gy, L, params[wn], prev=(*saved[P.name], P.pmode),
                                      wd=_wp(packs, L.name, 1), ypool=saved.get(L.name + ".pool_in"))
        elif need_gx:
            B, H, W, _ = gy.shape
            gx = _empty(B, 1, H, W, like=gy)
            N.call("ebsdvae_conv3x3_cout1_fwd", N.ptr(gy), None, ACT_RAW, N.ptr(params[wn]), None,
                   N.ptr(gx), 1, B, H, W, L.cout, N.stream())
    return out, gx


def encode_latents(plan: Plan, x, params, packs=None):
    """Encoder-only inference (BASELINE c4, build_dictionary): x (B,1,S,S) -> mu (B,L)."""
    enc, _ = encoder_forward(plan, x, params, packs=packs, train=False)
    B = x.shape[0]
    mu = _empty(B, plan.latent_dim, like=x)
    work = _heads_work(B, plan, x)
    N.call("ebsdvae_latent_mu", N.ptr(enc), N.ptr(params["mu.0.weight"]), N.ptr(params["mu.0.bias"]),
           N.ptr(mu), N.ptr(work), B, plan.enc_channels, plan.enc_side, plan.latent_dim, N.stream())
    return mu


# ----------------------------------------------------------------------------- heads
HEAD_NAMES = ("mu.0.weight", "mu.0.bias", "logvar.0.weight", "logvar.0.bias",
              "linear2.0.weight", "linear2.0.bias")


def _heads_work(B, plan: Plan, like):
    """Split-K scratch of the heads launches (ebsdvae_heads_work bytes; stream-ordered reuse
    through torch's caching allocator)."""
    nbytes = N.call("ebsdvae_heads_work", B, plan.enc_channels, plan.enc_side, plan.latent_dim)
    if nbytes <= 0:
        raise RuntimeError(f"heads: unsupported shape C={plan.enc_channels} S={plan.enc_side} "
                           f"L={plan.latent_dim}")
    return _scratch(nbytes // 4, device=like.device)


def heads_forward(plan: Plan, enc, params, eps):
    B = enc.shape[0]
    L, F = plan.latent_dim, plan.feat
    s, C = plan.enc_side, plan.enc_channels
    flat = _empty(B, F, like=enc)
    mu = _empty(B, L, like=enc)
    std = _empty(B, L, like=enc)
    z = _empty(B, L, like=enc)
    dec_in = _empty(B, s, s, C, like=enc)
    work = _heads_work(B, plan, enc)
    N.call("ebsdvae_heads_fwd", N.ptr(enc), *[N.ptr(params[n]) for n in HEAD_NAMES], N.ptr(eps),
           N.ptr(flat), N.ptr(mu), N.ptr(std), N.ptr(z), N.ptr(dec_in), N.ptr(work), B, C, s, L,
           N.stream())
    return flat, mu, std, z, dec_in


def heads_backward(plan: Plan, g_dec, g_z, g_mu, g_std, flat, std, z, eps, params, grads=None):
    B = g_dec.shape[0]
    L, F = plan.latent_dim, plan.feat
    s, C = plan.enc_side, plan.enc_channels
    g_enc = _empty(B, s, s, C, like=g_dec)
    gs = _empty(B, 2 * L + F, like=g_dec)
    N.call("ebsdvae_heads_bwd", N.ptr(g_dec), N.ptr(g_z), N.ptr(g_mu), N.ptr(g_std), N.ptr(std),
           N.ptr(eps), N.ptr(params["mu.0.weight"]), N.ptr(params["logvar.0.weight"]),
           N.ptr(params["linear2.0.weight"]), N.ptr(g_enc), N.ptr(gs), N.ptr(_heads_work(B, plan, g_dec)),
           B, C, s, L, N.stream())
    out = {n: _grad_buf(grads, n, params[n]) for n in HEAD_NAMES}
    # the heads' weight gradients are off the critical path (g_enc is all the encoder
    # backward needs): on the side stream inside deferred_side_join() (the trainer's step)
    side = _side_stream(g_dec.device) if _DEFER else None
    ctx = contextlib.nullcontext()
    if side is not None:
        side = _side_use(g_dec.device, flat, z, gs)
        ctx = torch.cuda.stream(side)
    with ctx:
        nbytes = N.call("ebsdvae_heads_wgrad_work", B, F, L)
        work = _scratch(nbytes // 4, device=g_dec.device)
        N.call("ebsdvae_heads_wgrad", N.ptr(flat), N.ptr(z), N.ptr(gs),
               *[N.ptr(out[n]) for n in HEAD_NAMES], N.ptr(work), B, F, L, N.stream())
    if side is not None:
        _KEEP[_dev_key(g_dec.device)].append(work)
    return g_enc, out


# ----------------------------------------------------------------------------- decoder
def decoder_forward(plan: Plan, dec_in, params, packs=None, final=True):
    """dec_in: (B,s,s,C) NHWC.  Returns (x_hat (B,1,S,S), saved).  final=False leaves out the
    final conv (x_hat None): the training step computes it in network_end."""
    B = dec_in.shape[0]
    saved = {"__dec_in__": dec_in}
    src, sst = dec_in, None
    for L in plan.dec:
        y, st = conv_forward(src, sst, L, params[L.name + ".weight"], params[L.name + ".bias"], B,
                             wp=_wp(packs, L.name, 0))
        saved[L.name] = (y, st)
        src, sst = y, st
    _record(plan.dec, saved)
    if not final:
        return None, saved
    S = plan.image_size
    x_hat = _empty(B, 1, S, S, like=dec_in)
    N.call("ebsdvae_conv3x3_cout1_fwd", N.ptr(src), N.ptr(sst), ACT_NORM,
           N.ptr(params["decoder.14.weight"]), N.ptr(params["decoder.14.bias"]), N.ptr(x_hat), 0,
           B, S, S, plan.inplanes, N.stream())
    return x_hat, saved


def decoder_backward(plan: Plan, g_xhat, saved, params, grads=None, packs=None, end=None):
    """g_xhat: (B,1,S,S).  Returns (grads dict, g_dec_in (B,s,s,C) NHWC).  The layers'
    weight-gradient reductions run batched when it returns.  end: the NetEnd of network_end
    (g_xhat None), whose pass already produced the last block's reduce sums and the final
    conv's gradient slices."""
    with batched_wgrad_reduce():
        return _decoder_backward(plan, g_xhat, saved, params, grads, packs, end)


def _decoder_backward(plan, g_xhat, saved, params, grads, packs, end=None):
    out = {}
    last = plan.dec[-1]
    y13, st13 = saved[last.name]
    B = y13.shape[0]
    S, p = plan.image_size, plan.inplanes
    wn, bn = "decoder.14.weight", "decoder.14.bias"
    dw = _grad_buf(grads, wn, params[wn])
    db = _grad_buf(grads, bn, params[bn])
    if end is not None:
        gy_last = in_backward_final_from(end, params[wn], y13, st13, dw, db)
    else:
        g1 = g_xhat.reshape(B, S, S)
        # last conv fused into the last block's InstanceNorm backward: its input gradient is
        # recomputed from g1 on the fly, its weight gradient accumulated in the reduce pass
        gy_last = in_backward_final(g1, params[wn], y13, st13, dw, db)
    out[wn], out[bn] = dw, db
    g_next, part = None, None
    for i in reversed(range(len(plan.dec))):
        L = plan.dec[i]
        y, st = saved[L.name]
        fk = False
        if i == len(plan.dec) - 1:
            gy = gy_last
        else:   # a summed upsample adjoint (conv_dgrad sum_up) arrives at y's resolution
            pm = P_ID if (L.pmode == P_UP and g_next.shape[1] == y.shape[1]) else L.pmode
            fk = fork_arm(y.device)   # the weight gradient below forks on the apply's completion
            gy = in_backward(g_next, pm, y, st, part=part)
        wn, bn = L.name + ".weight", L.name + ".bias"
        src, sst = (saved["__dec_in__"], None) if i == 0 else saved[plan.dec[i - 1].name]
        dw = _grad_buf(grads, wn, params[wn])
        db = _grad_buf(grads, bn, params[bn])
        if _DWFUSE and i > 0 and L.src_mode in (ACT_NORM, ACT_NORM_UP) and \
                dwgrad_ok(gy, L, _wp(packs, L.name, 1), L.src_mode, plan.dec[i - 1].pmode):
            # input + weight gradient in one pass (the last block's gy has no side-stream fork)
            g_next, part = conv_dwgrad(gy, L, _wp(packs, L.name, 1), src, sst, L.src_mode, dw, db)
            out[wn], out[bn] = dw, db
            continue
        conv_wgrad(src, sst, L.src_mode, gy, L.cin, L.cout, L.kind, dw, db, fork=fk)
        out[wn], out[bn] = dw, db
        if i > 0:
            P = plan.dec[i - 1]
            g_next, part = conv_dgrad(gy, L, params[wn], prev=(*saved[P.name], P.pmode),
                                      wd=_wp(packs, L.name, 1), sum_up=True)
        else:
            g_next = conv_dgrad(gy, L, params[wn], wd=_wp(packs, L.name, 1))
    s, C = plan.enc_side, plan.enc_channels
    g_dec = _empty(B, s, s, C, like=y13)
    N.call("ebsdvae_upsample2_bwd", N.ptr(g_next), N.ptr(g_dec), B, s, s, C, N.stream())
    return out, g_dec


# ----------------------------------------------------------------------------- loss
def loss_forward(x_hat, x, z, mu, std, kl_lambda: float):
    """Returns (loss, kl_loss, recon_loss) 0-d tensors and per-sample (elbo, kl, recon).
    Inside deferred_side_join() it runs on the side stream: the loss backward does not read
    the loss values, so they are off the critical path (ready at the block's join)."""
    B = x_hat.shape[0]
    P = x_hat[0].numel()
    L = z.shape[1]
    # outputs allocated on the current stream (the caller's), written on the side stream and
    # kept alive until the join
    elbo, kl, recon = _empty(B, like=x_hat), _empty(B, like=x_hat), _empty(B, like=x_hat)
    loss, kl_loss, recon_loss = (_scratch(device=x_hat.device)
                                 for _ in range(3))
    side = _side_stream(x_hat.device) if _DEFER else None
    ctx = contextlib.nullcontext()
    if side is not None:
        side = _side_use(x_hat.device, x_hat, x, z, mu, std, elbo, kl, recon, loss, kl_loss,
                         recon_loss)
        ctx = torch.cuda.stream(side)
    with ctx:
        N.call("ebsdvae_vae_loss_fwd", N.ptr(x_hat), N.ptr(x), N.ptr(z), N.ptr(mu), N.ptr(std),
               float(kl_lambda), N.ptr(elbo), N.ptr(kl), N.ptr(recon), N.ptr(loss), N.ptr(kl_loss),
               N.ptr(recon_loss), B, P, L, N.stream())
    return (loss, kl_loss, recon_loss), (elbo, kl, recon)


def loss_forward_parts(end: NetEnd, z, mu, std, kl_lambda: float, P: int):
    """loss_forward with the BCE sums of network_end (same outputs, same side-stream rule)."""
    B, L = z.shape
    elbo, kl, recon = _empty(B, like=z), _empty(B, like=z), _empty(B, like=z)
    loss, kl_loss, recon_loss = (_scratch(device=z.device)
                                 for _ in range(3))
    side = _side_stream(z.device) if _DEFER else None
    ctx = contextlib.nullcontext()
    if side is not None:
        side = _side_use(z.device, end.bce, z, mu, std, elbo, kl, recon, loss, kl_loss, recon_loss)
        ctx = torch.cuda.stream(side)
    with ctx:
        N.call("ebsdvae_vae_loss_fwd_parts", N.ptr(end.bce), end.tiles, N.ptr(z), N.ptr(mu),
               N.ptr(std), float(kl_lambda), N.ptr(elbo), N.ptr(kl), N.ptr(recon), N.ptr(loss),
               N.ptr(kl_loss), N.ptr(recon_loss), B, P, L, N.stream())
    return (loss, kl_loss, recon_loss), (elbo, kl, recon)


def loss_backward(x_hat, x, z, mu, std, kl_lambda: float, g_loss=None, g_kl=None, g_recon=None,
                  g_elbo=None, scale: float = 1.0, need_gx=False, out=None, P: int | None = None):
    """x_hat None (with P the pixels per pattern): only the KL gradients (network_end made the
    logit gradient); g_xhat is then None."""
    if x_hat is None:
        B, L = z.shape
        g_z, g_mu, g_std = _empty_like(z), _empty_like(mu), _empty_like(std)
        N.call("ebsdvae_vae_loss_bwd", None, None, N.ptr(z), N.ptr(mu), N.ptr(std),
               float(kl_lambda), N.ptr(g_loss), N.ptr(g_kl), N.ptr(g_recon), N.ptr(g_elbo),
               float(scale), None, N.ptr(g_z), N.ptr(g_mu), N.ptr(g_std), None, B, P, L, N.stream())
        return None, g_z, g_mu, g_std, None
    """Gradients of the loss outputs w.r.t. (x_hat, z, mu, std[, x]).  `out` may supply the
    four destination tensors (persistent buffers for graph capture)."""
    B = x_hat.shape[0]
    P = x_hat[0].numel()
    L = z.shape[1]
    if out is None:
        out = (_empty_like(x_hat), _empty_like(z), _empty_like(mu),
               _empty_like(std))
    g_xhat, g_z, g_mu, g_std = out
    g_x = _empty_like(x) if need_gx else None
    N.call("ebsdvae_vae_loss_bwd", N.ptr(x_hat), N.ptr(x), N.ptr(z), N.ptr(mu), N.ptr(std),
           float(kl_lambda), N.ptr(g_loss), N.ptr(g_kl), N.ptr(g_recon), N.ptr(g_elbo),
           float(scale), N.ptr(g_xhat), N.ptr(g_z), N.ptr(g_mu), N.ptr(g_std), N.ptr(g_x),
           B, P, L, N.stream())
    return g_xhat, g_z, g_mu, g_std, g_x


def normal_(out, seed: int, offset: int = 0, counter=None):
    """Fill `out` with N(0,1) draws (Philox).  `counter`: optional device uint64 tensor
    (int64 dtype) bumped on every call, for graph-replayed sampling."""
    cptr = None
    if counter is not None:
        if not counter.is_cuda or counter.dtype != torch.int64:
            raise TypeError("counter must be a device int64 tensor")
        cptr = counter.data_ptr()
    N.call("ebsdvae_normal_fill", N.ptr(out), out.numel(), seed & (2 ** 64 - 1),
           offset & (2 ** 64 - 1), cptr, N.stream())
    return out
