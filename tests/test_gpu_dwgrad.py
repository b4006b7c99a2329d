"""The fused input + weight gradient of the 32 -> 32 layers (csrc/conv_fused.hip,
ebsdvae_conv3x3_dwgrad_f16; encoder.1 and decoder.13 of the training step) against the float64
oracle: the input gradient with the previous block's fused InstanceNorm-backward reduce (h, and
the block's gy after the apply), the summed upsample adjoint for decoder.13, the weight and bias
gradients -- at the f16x3 tolerance, with the gradient operand at 1e-7 scale, images 1e3 apart
and weight scales 1e-5 ... 100, as the separate kernels are tested (tests/test_gpu_kernels.py)."""
import numpy as np
import pytest
import torch

from latice import _native as N
from latice import engine as E
from oracle import vae_oracle as O
from test_gpu_kernels import SPLIT_TOL, _pack_f16_dgrad, act_oracle, dev, h_oracle, host

pytestmark = pytest.mark.gpu

CASES = [  # (H, layer kind, source mode, routing of the previous block)
    (128, E.KIND_CONV, E.ACT_NORM, E.P_ID),       # encoder.1 at c2
    (128, E.KIND_CONVT, E.ACT_NORM_UP, E.P_UP),   # decoder.13 at c2
    (256, E.KIND_CONV, E.ACT_NORM, E.P_ID),       # encoder.1 at c5
    (64, E.KIND_CONVT, E.ACT_NORM_UP, E.P_UP),
]


@pytest.mark.parametrize("wscale", [0.1, 1e-5, 100.0])
@pytest.mark.parametrize("gscale", [1.0, 1e-7])
@pytest.mark.parametrize("H,kind,mode,pmode", CASES)
def test_fused_dgrad_wgrad_matches_oracle(cuda, H, kind, mode, pmode, gscale, wscale):
    C = 32
    B = 3 if H <= 128 else 2
    rng = np.random.default_rng(11 + H + kind + int(np.log10(wscale)) + int(gscale < 1))
    Hs = H if pmode == E.P_ID else H // 2
    y = rng.standard_normal((B, Hs, Hs, C)) * 2 + 0.5
    xh, mean, rstd = O.instance_norm(y)
    st = np.stack([mean[:, 0, 0, :], rstd[:, 0, 0, :]], -1)
    gy = rng.standard_normal((B, H, H, C)) * gscale
    gy[1] *= 1e3
    wc = rng.standard_normal((C, C, 3, 3)) * wscale               # conv-equivalent (co, ci, 3, 3)
    wparam = wc if kind == E.KIND_CONV else wc.transpose(1, 0, 2, 3)[:, :, ::-1, ::-1].copy()
    layer = E.ConvLayer("t", kind, C, C, H, mode, 0)
    dw = torch.empty(wparam.shape, device="cuda")
    db = torch.empty(C, device="cuda")
    with E.precision("f16x3"):
        y_d, st_d = dev(y), dev(st)
        wd = _pack_f16_dgrad(dev(wparam), layer)
        g_d = dev(gy)
        g_d.ev_gmax = dev(np.abs(gy).reshape(B, -1).max(1, keepdims=True))
        assert E.dwgrad_ok(g_d, layer, wd, mode, pmode)
        with E.record_launches() as launched:
            gin, part = E.conv_dwgrad(g_d, layer, wd, y_d, st_d, mode, dw, db)
        g_prev = E.in_backward(gin, E.P_ID, y_d, st_d, part=part)
    assert "ebsdvae_conv3x3_dwgrad_f16" in launched
    a = act_oracle(y, mean, rstd, mode)
    gn = O.conv3x3_dgrad(gy, wc)
    hn = h_oracle(gn, xh, pmode, summed=pmode == E.P_UP)
    ga = O.upsample2_bwd(gn) if pmode == E.P_UP else gn
    ref = O.instance_norm_bwd(ga * O.lrelu_slope(xh), xh, rstd)
    for b in range(B):   # per image: image 1 is 1e3 larger
        assert O.rel_err(host(gin)[b], hn[b]) < SPLIT_TOL["f16x3"], b
        assert O.rel_err(host(g_prev)[b], ref[b]) < 2e-4, b
    rw, rb = O.conv3x3_wgrad(a, gy)
    if kind == E.KIND_CONVT:
        rw = rw.transpose(1, 0, 2, 3)[:, :, ::-1, ::-1]
    assert O.rel_err(host(dw), rw) < SPLIT_TOL["f16x3"]
    assert O.rel_err(host(db), rb) < 5e-5


def test_fused_dgrad_wgrad_shape_queries(cuda):
    assert N.call("ebsdvae_conv3x3_dwgrad_slices", 256, 128, 128, 32, 32) == 256
    assert N.call("ebsdvae_conv3x3_dwgrad_stat_tiles", 128, 128) == 256
    assert N.call("ebsdvae_conv3x3_dwgrad_slices", 4, 128, 128, 64, 32) == -1
    assert N.call("ebsdvae_conv3x3_dwgrad_slices", 4, 96, 96, 32, 32) == -1   # 12 tiles: not 2^k
