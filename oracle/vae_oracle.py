"""ORACLE — test infrastructure only (never imported by the product path).

A float64 numpy restatement of the reference VAE hot path, forward AND an
explicitly derived backward, in the same decomposition the HIP kernels use
(NHWC activations, 3x3 convs as 9 shifted GEMMs, InstanceNorm as plane
statistics + normalise, LeakyReLU, 2x2 max-pool with first-max-wins argmax,
nearest x2 upsample, heads, reparameterisation, BCE-with-logits + Monte-Carlo KL).

It is pinned against the golden vectors in tests/golden/*.npz, which were produced
by running the reference itself (tests/golden/make_golden.py) under torch
autograd, so both the forward algebra and the hand-derived gradient formulas are
checked against the reference before this module is trusted as a checker.

Reference anchors (all in /root/reference):
  * model structure        latice/model.py:90-150
  * forward / flatten      latice/model.py:40-66   (flatten(1,-1) in NCHW order)
  * reparameterise         latice/model.py:25-38   (std = exp(logvar/2); z = mu + eps*std)
  * conv block             latice/model.py:93-98   (Conv2d 3x3 s1 p1 -> InstanceNorm2d(eps 1e-5,
                                                     affine False) -> LeakyReLU(0.02))
  * conv-transpose block   latice/model.py:100-107 (ConvTranspose2d 3x3 s1 p1 == conv with the
                                                     weight transposed and spatially flipped)
  * max-pool / upsample    latice/model.py:112-124, 134-146
  * BCE-with-logits        latice/lightning_module.py:79-92
  * Monte-Carlo KL         latice/lightning_module.py:94-120
  * compute_loss           latice/lightning_module.py:122-156
"""
from __future__ import annotations

import numpy as np

LRELU_SLOPE = 0.02     # latice/model.py:97,106
IN_EPS = 1e-5          # nn.InstanceNorm2d default, latice/model.py:96,105

ENC_IDX = (0, 1, 3, 4, 6, 7, 9, 10, 12, 13)      # latice/model.py:109-125
POOL_AFTER = (1, 3, 5, 7, 9)                       # positions in ENC_IDX followed by MaxPool2d
DEC_IDX = (1, 2, 4, 5, 7, 8, 10, 11, 13)          # latice/model.py:133-148
UP_BEFORE = (0, 2, 4, 6, 8)                        # positions in DEC_IDX preceded by an Upsample


# ----------------------------------------------------------------------------- primitives
def conv_w_from_convT(wT: np.ndarray) -> np.ndarray:
    """ConvTranspose2d(Ci,Co,3,s1,p1) weight (Ci,Co,3,3) -> equivalent Conv2d weight (Co,Ci,3,3)."""
    return np.ascontiguousarray(wT.transpose(1, 0, 2, 3)[:, :, ::-1, ::-1])


def conv3x3(x: np.ndarray, w: np.ndarray, b: np.ndarray) -> np.ndarray:
    """NHWC 3x3 stride-1 pad-1 cross-correlation: y = b + sum_tap xpad[shift] @ W_tap."""
    n, h, wd, ci = x.shape
    xp = np.zeros((n, h + 2, wd + 2, ci), x.dtype)
    xp[:, 1:-1, 1:-1] = x
    y = np.broadcast_to(b.astype(x.dtype), (n, h, wd, w.shape[0])).copy()
    for kh in range(3):
        for kw in range(3):
            y += xp[:, kh:kh + h, kw:kw + wd, :] @ w[:, :, kh, kw].T.astype(x.dtype)
    return y


def conv3x3_dgrad(g: np.ndarray, w: np.ndarray) -> np.ndarray:
    n, h, wd, co = g.shape
    ci = w.shape[1]
    gp = np.zeros((n, h + 2, wd + 2, ci), g.dtype)
    for kh in range(3):
        for kw in range(3):
            gp[:, kh:kh + h, kw:kw + wd, :] += g @ w[:, :, kh, kw].astype(g.dtype)
    return gp[:, 1:-1, 1:-1]


def conv3x3_wgrad(x: np.ndarray, g: np.ndarray):
    n, h, wd, ci = x.shape
    co = g.shape[-1]
    xp = np.zeros((n, h + 2, wd + 2, ci), x.dtype)
    xp[:, 1:-1, 1:-1] = x
    dw = np.zeros((co, ci, 3, 3), x.dtype)
    g2 = g.reshape(-1, co)
    for kh in range(3):
        for kw in range(3):
            dw[:, :, kh, kw] = g2.T @ xp[:, kh:kh + h, kw:kw + wd, :].reshape(-1, ci)
    return dw, g2.sum(0)


def instance_norm(y: np.ndarray):
    """Per-(n,c) plane statistics, biased variance (InstanceNorm2d, affine=False)."""
    mean = y.mean(axis=(1, 2), keepdims=True)
    var = ((y - mean) ** 2).mean(axis=(1, 2), keepdims=True)
    rstd = 1.0 / np.sqrt(var + IN_EPS)
    return (y - mean) * rstd, mean, rstd


def instance_norm_bwd(gxh: np.ndarray, xh: np.ndarray, rstd: np.ndarray) -> np.ndarray:
    m1 = gxh.mean(axis=(1, 2), keepdims=True)
    m2 = (gxh * xh).mean(axis=(1, 2), keepdims=True)
    return rstd * (gxh - m1 - xh * m2)


def lrelu(v):
    return np.where(v > 0, v, LRELU_SLOPE * v)


def lrelu_slope(v):
    return np.where(v > 0, 1.0, LRELU_SLOPE)


def maxpool2(a: np.ndarray):
    """2x2/2 max-pool; returns pooled values and the argmax slot 0..3 (row-major window,
    first maximum wins like ATen's CPU kernel)."""
    n, h, w, c = a.shape
    win = a.reshape(n, h // 2, 2, w // 2, 2, c).transpose(0, 1, 3, 2, 4, 5).reshape(n, h // 2, w // 2, 4, c)
    arg = np.argmax(win, axis=3)          # numpy argmax also returns the first maximum
    return np.take_along_axis(win, arg[:, :, :, None, :], 3)[:, :, :, 0, :], arg


def maxpool2_bwd(g: np.ndarray, arg: np.ndarray) -> np.ndarray:
    n, h2, w2, c = g.shape
    out = np.zeros((n, h2, w2, 4, c), g.dtype)
    np.put_along_axis(out, arg[:, :, :, None, :], g[:, :, :, None, :], 3)
    return out.reshape(n, h2, w2, 2, 2, c).transpose(0, 1, 3, 2, 4, 5).reshape(n, 2 * h2, 2 * w2, c)


def upsample2(a: np.ndarray) -> np.ndarray:
    return a.repeat(2, axis=1).repeat(2, axis=2)


def upsample2_bwd(g: np.ndarray) -> np.ndarray:
    n, h, w, c = g.shape
    return g.reshape(n, h // 2, 2, w // 2, 2, c).sum(axis=(2, 4))


def nchw_flatten(a_nhwc: np.ndarray) -> np.ndarray:
    """encoder_out.flatten(1,-1) of the NCHW tensor (latice/model.py:57-58): index c*HW + h*W + w."""
    return a_nhwc.transpose(0, 3, 1, 2).reshape(a_nhwc.shape[0], -1)


def nchw_unflatten(f: np.ndarray, c: int, s: int) -> np.ndarray:
    """out.view(encoder_out.size()) (latice/model.py:64) then to NHWC."""
    return f.reshape(f.shape[0], c, s, s).transpose(0, 2, 3, 1)


# ----------------------------------------------------------------------------- model
def _params(sd, dtype):
    return {k: np.asarray(v, dtype) for k, v in sd.items()}


def forward(sd, x_nchw: np.ndarray, eps: np.ndarray, dtype=np.float64):
    """Full forward. Returns (outputs dict, cache for backward).  dtype=np.float32 runs the
    same algorithm in single precision (used to measure generic fp32 noise)."""
    p = _params(sd, dtype)
    x = np.asarray(x_nchw, dtype).transpose(0, 2, 3, 1)
    cache = {"x": x, "enc": [], "dec": []}
    a = x
    for i, idx in enumerate(ENC_IDX):
        w, b = p[f"encoder.{idx}.0.weight"], p[f"encoder.{idx}.0.bias"]
        y = conv3x3(a, w, b)
        xh, mean, rstd = instance_norm(y)
        act = lrelu(xh)
        ent = {"a_in": a, "w": w, "xh": xh, "rstd": rstd, "y": y, "mean": mean}
        if i in POOL_AFTER:
            act, arg = maxpool2(act)
            ent["arg"] = arg
        cache["enc"].append(ent)
        a = act
    c, s = a.shape[-1], a.shape[1]
    flat = nchw_flatten(a)
    mu = flat @ p["mu.0.weight"].T + p["mu.0.bias"]
    logvar = flat @ p["logvar.0.weight"].T + p["logvar.0.bias"]
    std = np.exp(logvar / 2)
    e = np.asarray(eps, dtype)
    z = mu + e * std
    out = z @ p["linear2.0.weight"].T + p["linear2.0.bias"]
    a = nchw_unflatten(out, c, s)
    cache.update(flat=flat, mu=mu, std=std, eps=e, z=z, c=c, s=s)
    for i, idx in enumerate(DEC_IDX):
        if i in UP_BEFORE:
            a = upsample2(a)
        wT, b = p[f"decoder.{idx}.0.weight"], p[f"decoder.{idx}.0.bias"]
        w = conv_w_from_convT(wT)
        y = conv3x3(a, w, b)
        xh, mean, rstd = instance_norm(y)
        cache["dec"].append({"a_in": a, "w": w, "xh": xh, "rstd": rstd, "y": y, "mean": mean})
        a = lrelu(xh)
    cache["last_in"] = a
    x_hat = conv3x3(a, p["decoder.14.weight"], p["decoder.14.bias"])
    cache["p"] = p
    outs = {"z": z, "x_hat": x_hat.transpose(0, 3, 1, 2), "mu": mu, "std": std,
            "enc_out": flat}
    return outs, cache


def vae_loss(x_hat_nchw, x_nchw, z, mu, std, kl_lambda):
    """latice/lightning_module.py:79-156 (BCEWithLogits mean over C,H,W; MC KL mean over latent)."""
    xh = np.asarray(x_hat_nchw, np.float64)
    y = np.asarray(x_nchw, np.float64)
    bce = (1.0 - y) * xh + np.logaddexp(0.0, -xh)
    recon = bce.reshape(bce.shape[0], -1).mean(1)
    kl = (0.5 * z ** 2 - 0.5 * ((z - mu) / std) ** 2 - np.log(std)).mean(-1) * kl_lambda
    elbo = kl + recon
    return {"loss": elbo.mean(), "kl_loss": kl.mean(), "recon_loss": recon.mean(), "elbo": elbo}


def pinned_routing(y, st, pool: bool):
    """The discrete backward decisions of one block, taken from a float32 run's saved
    pre-norm output y (B,H,W,C) and statistics st (B,C,2) = {mean, rstd}, evaluated exactly
    as the HIP backward evaluates them (csrc/instnorm.hip in_bwd_kernel, conv_common.h
    inbwd_acc): xhat = (y - mean) * rstd in float32, LeakyReLU slope 1 where xhat > 0 (the
    fused reduce tests y > mean, the same predicate for rstd > 0), and
    for a max-pooled block the FIRST maximum of lrelu(xhat) = max(xhat, 0.02 xhat) in window
    order (0,0),(0,1),(1,0),(1,1) (ATen's CPU max_pool2d rule, latice/model.py:112-124).

    Routing is the only discontinuous part of the backward: max-pool argmax near-ties and
    LeakyReLU sign flips at xhat ~ 0 send gradient down different branches in any two
    evaluations that differ by rounding, so a float64 oracle is compared with a float32
    run on the SAME branches (see backward(pins=...))."""
    y = np.asarray(y, np.float32)
    st = np.asarray(st, np.float32)
    xh = (y - st[:, None, None, :, 0]) * st[:, None, None, :, 1]
    pos = xh > 0
    arg = None
    if pool:
        _, arg = maxpool2(np.maximum(xh, np.float32(LRELU_SLOPE) * xh))
    return pos, arg


def pins_from_blocks(enc_blocks, dec_blocks):
    """{("enc", i) / ("dec", i): pinned_routing(...)} from the (y, st) of every encoder block
    (ENC_IDX order) and decoder block (DEC_IDX order) of one float32 run."""
    pins = {("enc", i): pinned_routing(y, st, i in POOL_AFTER) for i, (y, st) in enumerate(enc_blocks)}
    pins.update({("dec", i): pinned_routing(y, st, False) for i, (y, st) in enumerate(dec_blocks)})
    return pins


def pins_from_cache(cache):
    """pins_from_blocks of an oracle run's own blocks (e.g. the float32 oracle)."""
    return pins_from_blocks(*blocks_from_cache(cache))


def forward_from_state(sd, x_nchw, eps, enc_blocks, dec_blocks):
    """State-pinned forward: the cache backward() needs, rebuilt in float64 from a float32
    run's saved block state -- its pre-norm conv outputs y and InstanceNorm statistics
    {mean, rstd} of every encoder block (ENC_IDX order) and decoder block (DEC_IDX order)
    -- instead of from this oracle's own forward.  Every other quantity (activations,
    pooling at the pinned argmax, heads, z, linear2, the final conv) is recomputed in
    float64 from that state with the same formulas as forward().  Returns (outs, cache,
    pins).

    Why: the forward is chaotic in a few places (an InstanceNorm over a near-constant
    plane, e.g. the saturated pattern of the vae128_b2_edge fixture, multiplies the
    rounding of y by rstd ~ 1e2), so two correct float32 runs can sit 1e-2 apart in weight
    gradient from float64 while their forwards agree to 1e-5.  Pinned to the run's own
    state, the only remaining difference is the backward arithmetic itself; the forward
    state is checked separately against the reference's golden outputs."""
    p = _params(sd, np.float64)
    x = np.asarray(x_nchw, np.float64).transpose(0, 2, 3, 1)
    pins = pins_from_blocks(enc_blocks, dec_blocks)
    cache = {"x": x, "enc": [], "dec": [], "p": p}

    def block(y, st):
        y = np.asarray(y, np.float64)
        st = np.asarray(st, np.float64)
        mean = st[:, None, None, :, 0]
        rstd = st[:, None, None, :, 1]
        return y, mean, rstd, (y - mean) * rstd

    def act(xh, pos):
        return np.where(pos, xh, LRELU_SLOPE * xh)

    a = x
    for i, idx in enumerate(ENC_IDX):
        y, mean, rstd, xh = block(*enc_blocks[i])
        pos, arg = pins[("enc", i)]
        ent = {"a_in": a, "w": p[f"encoder.{idx}.0.weight"], "xh": xh, "rstd": rstd, "y": y,
               "mean": mean}
        a = act(xh, pos)
        if i in POOL_AFTER:
            n, h, w, c = a.shape
            win = a.reshape(n, h // 2, 2, w // 2, 2, c).transpose(0, 1, 3, 2, 4, 5).reshape(n, h // 2, w // 2, 4, c)
            a = np.take_along_axis(win, arg[:, :, :, None, :], 3)[:, :, :, 0, :]
            ent["arg"] = arg
        cache["enc"].append(ent)
    c, s = a.shape[-1], a.shape[1]
    flat = nchw_flatten(a)
    mu = flat @ p["mu.0.weight"].T + p["mu.0.bias"]
    std = np.exp((flat @ p["logvar.0.weight"].T + p["logvar.0.bias"]) / 2)
    e = np.asarray(eps, np.float64)
    z = mu + e * std
    a = nchw_unflatten(z @ p["linear2.0.weight"].T + p["linear2.0.bias"], c, s)
    cache.update(flat=flat, mu=mu, std=std, eps=e, z=z, c=c, s=s)
    for i, idx in enumerate(DEC_IDX):
        if i in UP_BEFORE:
            a = upsample2(a)
        y, mean, rstd, xh = block(*dec_blocks[i])
        cache["dec"].append({"a_in": a, "w": conv_w_from_convT(p[f"decoder.{idx}.0.weight"]),
                             "xh": xh, "rstd": rstd, "y": y, "mean": mean})
        a = act(xh, pins[("dec", i)][0])
    cache["last_in"] = a
    x_hat = conv3x3(a, p["decoder.14.weight"], p["decoder.14.bias"])
    outs = {"z": z, "x_hat": x_hat.transpose(0, 3, 1, 2), "mu": mu, "std": std, "enc_out": flat}
    return outs, cache, pins


def blocks_from_cache(cache):
    """(enc_blocks, dec_blocks) = [(y, st)] of an oracle run (e.g. the float32 oracle)."""
    def blocks(key):
        return [(e["y"], np.stack([e["mean"][:, 0, 0, :], e["rstd"][:, 0, 0, :]], -1))
                for e in cache[key]]
    return blocks("enc"), blocks("dec")


def backward(cache, x_nchw, kl_lambda, g_loss: float = 1.0, pins=None, absum=None):
    """Gradients of compute_loss(...)['loss'] w.r.t. every parameter (state_dict names).

    pins (optional): {("enc"|"dec", i): (pos, arg)} from pinned_routing -- the LeakyReLU
    branch and max-pool argmax of block i are taken from there instead of from this
    evaluation's own float64 activations (decision-pinned oracle).
    absum (optional dict): filled with, per conv bias feeding an InstanceNorm (whose gradient
    sum_{b,h,w} gy is analytically zero), A_c = sum_{b,h,w} |gy| per channel -- the scale of
    an fp32 run's rounding residue on that zero (tests/pinned.py)."""
    pins = pins or {}
    p = cache["p"]
    grads = {}
    x = cache["x"]
    bsz = x.shape[0]
    xh_last = conv3x3(cache["last_in"], p["decoder.14.weight"], p["decoder.14.bias"])
    npx = xh_last.shape[1] * xh_last.shape[2]
    sig = 1.0 / (1.0 + np.exp(-xh_last))
    g = g_loss * (sig - x) / (npx * bsz)                       # d loss / d x_hat (NHWC, C=1)
    dw, db = conv3x3_wgrad(cache["last_in"], g)
    grads["decoder.14.weight"], grads["decoder.14.bias"] = dw, db
    ga = conv3x3_dgrad(g, p["decoder.14.weight"])
    for i in reversed(range(len(DEC_IDX))):
        idx = DEC_IDX[i]
        ent = cache["dec"][i]
        pin = pins.get(("dec", i))
        gxh = ga * (lrelu_slope(ent["xh"]) if pin is None else np.where(pin[0], 1.0, LRELU_SLOPE))
        gy = instance_norm_bwd(gxh, ent["xh"], ent["rstd"])
        dw, db = conv3x3_wgrad(ent["a_in"], gy)
        # conv weight (Co,Ci,kh,kw) = wT[ci,co,2-kh,2-kw]  =>  d wT = transpose/flip back
        grads[f"decoder.{idx}.0.weight"] = np.ascontiguousarray(dw.transpose(1, 0, 2, 3)[:, :, ::-1, ::-1])
        grads[f"decoder.{idx}.0.bias"] = db
        if absum is not None:
            absum[f"decoder.{idx}.0.bias"] = np.abs(gy).sum(axis=(0, 1, 2))
        ga = conv3x3_dgrad(gy, ent["w"])
        if i in UP_BEFORE:
            ga = upsample2_bwd(ga)
    # heads + reparameterisation + KL
    z, mu, std, e, flat = cache["z"], cache["mu"], cache["std"], cache["eps"], cache["flat"]
    lat = z.shape[1]
    kscale = g_loss * kl_lambda / (bsz * lat)
    g_out = nchw_flatten(ga)                                    # grad wrt linear2 output
    grads["linear2.0.weight"] = g_out.T @ z
    grads["linear2.0.bias"] = g_out.sum(0)
    gz = g_out @ p["linear2.0.weight"] + kscale * (z - (z - mu) / std ** 2)
    gmu = gz + kscale * ((z - mu) / std ** 2)
    gstd = kscale * ((z - mu) ** 2 / std ** 3 - 1.0 / std)
    glv = (gstd + gz * e) * std / 2.0
    grads["mu.0.weight"], grads["mu.0.bias"] = gmu.T @ flat, gmu.sum(0)
    grads["logvar.0.weight"], grads["logvar.0.bias"] = glv.T @ flat, glv.sum(0)
    gflat = gmu @ p["mu.0.weight"] + glv @ p["logvar.0.weight"]
    ga = nchw_unflatten(gflat, cache["c"], cache["s"])
    for i in reversed(range(len(ENC_IDX))):
        idx = ENC_IDX[i]
        ent = cache["enc"][i]
        pin = pins.get(("enc", i))
        if "arg" in ent:
            ga = maxpool2_bwd(ga, ent["arg"] if pin is None else pin[1])
        gxh = ga * (lrelu_slope(ent["xh"]) if pin is None else np.where(pin[0], 1.0, LRELU_SLOPE))
        gy = instance_norm_bwd(gxh, ent["xh"], ent["rstd"])
        dw, db = conv3x3_wgrad(ent["a_in"], gy)
        grads[f"encoder.{idx}.0.weight"], grads[f"encoder.{idx}.0.bias"] = dw, db
        if absum is not None:
            absum[f"encoder.{idx}.0.bias"] = np.abs(gy).sum(axis=(0, 1, 2))
        if i > 0:
            ga = conv3x3_dgrad(gy, ent["w"])
    return grads


def load_fixture(path: str):
    """Load a golden .npz (numpy, allow_pickle=False) and decode its inputs."""
    f = dict(np.load(path, allow_pickle=False))
    f["x"] = (f["x_u8"].astype(np.float32) / np.float32(255.0)).astype(np.float32)
    return f


def rel_err(a, b) -> float:
    """Norm-wise relative error max|a-b| / max|b|."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = max(np.abs(b).max(), 1e-30)
    return float(np.abs(a - b).max() / den)
