"""Debug: where the fused dgrad+wgrad (UPS form) differs from the oracle (error map by window
position within the 4x4 windows of a tile and by image)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ebsd-vae_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import torch
from latice import engine as E
from oracle import vae_oracle as O
from test_gpu_kernels import _pack_f16_dgrad, dev, h_oracle, host

H, C, B = int(sys.argv[1]) if len(sys.argv) > 1 else 128, 32, int(sys.argv[3]) if len(sys.argv) > 3 else 3
kind = int(sys.argv[2]) if len(sys.argv) > 2 else 1
ups = kind == 1
rng = np.random.default_rng(5)
Hs = H // 2 if ups else H
y = rng.standard_normal((B, Hs, Hs, C)) * 2 + 0.5
xh, mean, rstd = O.instance_norm(y)
st = np.stack([mean[:, 0, 0, :], rstd[:, 0, 0, :]], -1)
gy = rng.standard_normal((B, H, H, C))
wc = rng.standard_normal((C, C, 3, 3)) * 0.1
wparam = wc if kind == 0 else wc.transpose(1, 0, 2, 3)[:, :, ::-1, ::-1].copy()
mode = E.ACT_NORM_UP if ups else E.ACT_NORM
layer = E.ConvLayer("t", kind, C, C, H, mode, 0)
dw = torch.empty(wparam.shape, device="cuda"); db = torch.empty(C, device="cuda")
with E.precision("f16x3"):
    wd = _pack_f16_dgrad(dev(wparam), layer)
    g_d = dev(gy); g_d.ev_gmax = dev(np.abs(gy).reshape(B, -1).max(1, keepdims=True))
    gin, part = E.conv_dwgrad(g_d, layer, wd, dev(y), dev(st), mode, dw, db)
gn = O.conv3x3_dgrad(gy, wc)
hn = h_oracle(gn, xh, E.P_UP if ups else E.P_ID, summed=ups)
d = np.abs(host(gin) - hn)
print("max err", d.max(), "max ref", np.abs(hn).max())
T = 4 if ups else 8
e = d.reshape(B, Hs // T, T, Hs // T, T, C)
print("by image", e.max(axis=(1, 2, 3, 4, 5)))
print("by row-in-tile", e.max(axis=(0, 1, 3, 4, 5)))
print("by col-in-tile", e.max(axis=(0, 1, 2, 3, 5)))
print("by channel", np.round(e.max(axis=(0, 1, 2, 3, 4)), 4))
print("by tile row", np.round(e.max(axis=(0, 2, 3, 4, 5))[:8], 4), "tile col", np.round(e.max(axis=(0, 1, 2, 4, 5))[:8], 4))
bad = np.argwhere(d > 1e-3 * np.abs(hn).max())
print("n bad", len(bad), "first", bad[:10])
# tiles of 8x8 at H (4x4 windows at H/2 for UPS): error per tile index t = b*per_img + ty*ntx + tx
ntx = H // 8
et = d.reshape(B, ntx, T, ntx, T, C).max(axis=(2, 4, 5))   # (B, ty, tx)
flat = et.reshape(-1)
bad_t = np.nonzero(flat > 1e-3 * np.abs(hn).max())[0]
print("bad tiles:", len(bad_t), "of", flat.size, "first", bad_t[:16])
S = N_SL = None
from latice import _native as NN
S = NN.call("ebsdvae_conv3x3_dwgrad_slices", B, H, H, 32, 32)
tps = (flat.size + S - 1) // S
print("slices", S, "tps", tps, "bad tile positions within slice", sorted(set((bad_t % tps).tolist()))[:20])
g = host(gin)
b, r, c = 0, 0, 12
print("got      ", np.round(g[b, r, c, :6], 4))
print("ref      ", np.round(hn[b, r, c, :6], 4))
print("ref c-4  ", np.round(hn[b, r, c - 4, :6], 4))
print("ref c+4  ", np.round(hn[b, r, c + 4, :6], 4))
print("ref r+1  ", np.round(hn[b, r + 1, c, :6], 4))
gs = O.upsample2_bwd(gn)
print("gsum ref ", np.round(gs[b, r, c, :6], 4))
ratio = g[b, :4, 12:16] / np.where(np.abs(hn[b, :4, 12:16]) > 1e-6, hn[b, :4, 12:16], 1)
print("ratio window (0..3, 12..15) ch0", np.round(ratio[..., 0], 3))
