"""Stand-alone timing of single conv launches through the C ABI (HIP events, one stream),
for kernel A/B work and short rocprofv3 --pmc passes.

    python tools/conv_micro.py [--reps 20] [--pieces 3] [--only fwd32]

Cases are the training step's dominant shapes at B=256: each prints
the average launch time and the algorithmic fp32-equivalent TFLOP/s.
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ebsd-vae_amd")]

import torch  # noqa: E402

from latice import _native as N  # noqa: E402
from latice.engine import ACT_NORM, ACT_NORM_POOL, ACT_NORM_UP, P_ID, P_POOL, P_UP  # noqa: E402

# name: (kind, H, cin, cout, src_mode / pmode)
CASES = {
    "fwd32": ("fwd", 128, 32, 32, ACT_NORM),
    "fwd64": ("fwd", 64, 64, 64, ACT_NORM),
    "fwd128": ("fwd", 32, 128, 128, ACT_NORM),
    "fwd128s16": ("fwd", 16, 128, 128, ACT_NORM),
    "fwd32to64p": ("fwd", 64, 32, 64, ACT_NORM_POOL),
    "fwd64to32u": ("fwd", 128, 64, 32, ACT_NORM_UP),
    "fwd32pool": ("fwdpool", 128, 32, 32, ACT_NORM),
    # encoder.1 with its source recomputed from x (ebsdvae_conv3x3_fwd_split_first): the first
    # conv's statistics only, no y0 read
    "fwd32poolx": ("fwdfirst", 128, 32, 32, ACT_NORM),
    "fwd64pool": ("fwdpool", 64, 64, 64, ACT_NORM),
    "fwd128pool": ("fwdpool", 32, 128, 128, ACT_NORM),
    "fwd32to64n": ("fwd", 64, 32, 64, ACT_NORM),
    "fwd128s8": ("fwd", 8, 128, 128, ACT_NORM),
    "dgrad128s8": ("dgrad", 8, 128, 128, P_ID),
    "fwd128s16": ("fwd", 16, 128, 128, ACT_NORM),
    "dgrad128s16": ("dgrad", 16, 128, 128, P_ID),
    "dgrad32": ("dgrad", 128, 32, 32, P_ID),
    "dgrad64": ("dgrad", 64, 64, 64, P_ID),
    "dgrad32u": ("dgrad", 128, 32, 32, P_UP),
    # the encoder's pool-fed layers' input gradients, fused reduce over the 2x2 windows of
    # the producer's y (P_POOL) or over its pooled raw output (P_ID, engine ypool)
    "dgrad32to64p": ("dgrad", 64, 32, 64, P_POOL),
    "dgrad32to64i": ("dgrad", 64, 32, 64, P_ID),
    "dgrad64to128p": ("dgrad", 32, 64, 128, P_POOL),
    "dgrad64to128i": ("dgrad", 32, 64, 128, P_ID),
    "dgrad128": ("dgrad", 32, 128, 128, P_ID),
    "wgrad32": ("wgrad", 128, 32, 32, ACT_NORM),
    "wgrad32u": ("wgrad", 128, 32, 32, ACT_NORM_UP),
    "wgrad64": ("wgrad", 64, 64, 64, ACT_NORM),
    "wgrad128": ("wgrad", 32, 128, 128, ACT_NORM),
    "wgrad128s16": ("wgrad", 16, 128, 128, ACT_NORM),
    "wgrad64to128": ("wgrad", 32, 64, 128, ACT_NORM),
    # fused input + weight gradient of the 32-channel layers (csrc/conv_fused.hip): encoder.1
    # (same-resolution source, P_ID reduce) and decoder.13 (upsampled source, summed adjoint)
    "dwgrad32": ("dwgrad", 128, 32, 32, ACT_NORM),
    "dwgrad32u": ("dwgrad", 128, 32, 32, ACT_NORM_UP),
}


def run(name, reps, pieces, B, warm=1.0):
    kind, H, cin, cout, mode = CASES[name]
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    s = N.stream()
    flops = 2.0 * B * H * H * cin * cout * 9
    w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) * 0.05
    bias = torch.zeros(cout, device=dev)
    if kind in ("fwd", "fwdpool", "fwdfirst"):
        Hs = 2 * H if mode == ACT_NORM_POOL else (H // 2 if mode == ACT_NORM_UP else H)
        src = torch.randn(B, Hs, Hs, cin if kind != "fwdfirst" else 1, device=dev, generator=g)
        w0 = torch.randn(cin, 1, 3, 3, device=dev, generator=g) * 0.3
        b0 = torch.zeros(cin, device=dev)
        st_out = torch.empty(B, cout, 2, device=dev)
        st = torch.stack([torch.zeros(B, cin, device=dev), torch.ones(B, cin, device=dev)], -1).contiguous()
        wp = torch.empty(N.call("ebsdvae_pack_split_bytes", cin, cout, pieces) // 4, device=dev)
        d = (N.PackDesc * 1)(N.PackDesc(w.data_ptr(), wp.data_ptr(), cin, cout, 0, 0))
        N.call("ebsdvae_pack_conv_weights_split", ctypes.addressof(d), 1, pieces, s)
        y = torch.empty(B, H, H, cout, device=dev)
        T = N.call("ebsdvae_conv3x3_split_stat_tiles", H, H, cout)
        part = torch.empty(B, T, cout, 2, device=dev)

        yp = torch.empty(B, H // 2, H // 2, cout, device=dev)

        def launch():
            if kind == "fwdfirst":
                N.call("ebsdvae_conv3x3_fwd_split_first", src.data_ptr(), st.data_ptr(), w0.data_ptr(),
                       b0.data_ptr(), wp.data_ptr(), bias.data_ptr(), y.data_ptr(), yp.data_ptr(),
                       part.data_ptr(), st_out.data_ptr(), B, H, H, cin, cout, pieces, s)
                return
            if kind == "fwdpool":
                N.call("ebsdvae_conv3x3_fwd_split_pooled", src.data_ptr(), st.data_ptr(), mode,
                       wp.data_ptr(), bias.data_ptr(), y.data_ptr(), yp.data_ptr(), part.data_ptr(),
                       B, H, H, cin, cout, pieces, s)
                return
            N.call("ebsdvae_conv3x3_fwd_split", src.data_ptr(), st.data_ptr(), mode, wp.data_ptr(),
                   bias.data_ptr(), y.data_ptr(), part.data_ptr(), None, B, H, H, cin, cout, pieces, s)
    elif kind == "dgrad":
        # input gradient of a cin->cout layer: a conv cout->cin, fused reduce of the block
        # feeding it (y_prev at 2H for P_POOL)
        gy = torch.randn(B, H, H, cout, device=dev, generator=g)
        Hp = 2 * H if mode == P_POOL else (H // 2 if mode == P_UP else H)
        yprev = torch.randn(B, Hp, Hp, cin, device=dev, generator=g)
        stp = torch.stack([torch.zeros(B, cin, device=dev), torch.ones(B, cin, device=dev)], -1).contiguous()
        wp = torch.empty(N.call("ebsdvae_pack_split_bytes", cout, cin, pieces) // 4, device=dev)
        d = (N.PackDesc * 1)(N.PackDesc(w.data_ptr(), wp.data_ptr(), cin, cout, 0, 1))
        N.call("ebsdvae_pack_conv_weights_split", ctypes.addressof(d), 1, pieces, s)
        gin = torch.empty(B, H, H, cin, device=dev)
        T = N.call("ebsdvae_conv3x3_split_stat_tiles", H, H, cin)
        part = torch.empty(B, T, cin, 2, dtype=torch.float64, device=dev)

        gmx = gy.abs().reshape(B, 4, -1).amax(2).contiguous()   # per-tile maxima (f16)

        def launch():
            if pieces == 16:
                N.call("ebsdvae_conv3x3_dgrad_inbwd_f16", gy.data_ptr(), gmx.data_ptr(), 4, wp.data_ptr(),
                       gin.data_ptr(), yprev.data_ptr(), stp.data_ptr(), mode, part.data_ptr(), B, H, H,
                       cout, cin, s)
                return
            N.call("ebsdvae_conv3x3_dgrad_inbwd_split", gy.data_ptr(), wp.data_ptr(), gin.data_ptr(),
                   yprev.data_ptr(), stp.data_ptr(), mode, part.data_ptr(), B, H, H, cout, cin, pieces, s)
    elif kind == "dwgrad":
        flops *= 2   # both contractions
        Hs = H // 2 if mode == ACT_NORM_UP else H
        src = torch.randn(B, Hs, Hs, cin, device=dev, generator=g)
        st = torch.stack([torch.zeros(B, cin, device=dev), torch.ones(B, cin, device=dev)], -1).contiguous()
        gy = torch.randn(B, H, H, cout, device=dev, generator=g)
        wp = torch.empty(N.call("ebsdvae_pack_split_bytes", cout, cin, 16) // 4, device=dev)
        d = (N.PackDesc * 1)(N.PackDesc(w.data_ptr(), wp.data_ptr(), cin, cout, 0, 1))
        N.call("ebsdvae_pack_conv_weights_split", ctypes.addressof(d), 1, 16, s)
        S_ = N.call("ebsdvae_conv3x3_dwgrad_slices", B, H, H, cin, cout)
        T = N.call("ebsdvae_conv3x3_dwgrad_stat_tiles", H, H)
        wpart = torch.empty(S_, 9, cout, cin, device=dev)
        bpart = torch.empty(S_, cout, device=dev)
        gin = torch.empty(B, Hs, Hs, cin, device=dev)
        part = torch.empty(B, T, cin, 2, dtype=torch.float64, device=dev)
        gmx = gy.abs().reshape(B, 4, -1).amax(2).contiguous()

        def launch():
            N.call("ebsdvae_conv3x3_dwgrad_f16", gy.data_ptr(), gmx.data_ptr(), 4, wp.data_ptr(),
                   src.data_ptr(), st.data_ptr(), mode, gin.data_ptr(), part.data_ptr(),
                   wpart.data_ptr(), bpart.data_ptr(), B, H, H, cin, cout, s)
    else:
        Hs = H // 2 if mode == ACT_NORM_UP else H
        src = torch.randn(B, Hs, Hs, cin, device=dev, generator=g)
        st = torch.stack([torch.zeros(B, cin, device=dev), torch.ones(B, cin, device=dev)], -1).contiguous()
        gy = torch.randn(B, H, H, cout, device=dev, generator=g)
        S_ = N.call("ebsdvae_conv3x3_wgrad_split_slices", B, H, H, cin, cout, pieces)
        wpart = torch.empty(S_, 9, cout, cin, device=dev)
        bpart = torch.empty(S_, cout, device=dev)

        gmx = gy.abs().reshape(B, 4, -1).amax(2).contiguous()

        def launch():
            if pieces == 16:
                N.call("ebsdvae_conv3x3_wgrad_f16", src.data_ptr(), st.data_ptr(), mode, gy.data_ptr(),
                       gmx.data_ptr(), 4, wpart.data_ptr(), bpart.data_ptr(), B, H, H, cin, cout, s)
                return
            N.call("ebsdvae_conv3x3_wgrad_split", src.data_ptr(), st.data_ptr(), mode, gy.data_ptr(),
                   wpart.data_ptr(), bpart.data_ptr(), B, H, H, cin, cout, pieces, s)
    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    t_end = time.time() + warm   # DVFS: let the clock settle under back-to-back launches
    while time.time() < t_end:
        for _ in range(10):
            launch()
        torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    lib = N.load()
    if hasattr(lib, "ebsdvae_debug_pipe_trace"):   # EV_PIPE_TRACE build: per-wave cycle split
        import numpy as np
        buf = np.zeros(4096 * 8 * 6, dtype=np.uint64)
        lib.ebsdvae_debug_pipe_trace(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(buf.nbytes))
        t = buf.reshape(4096, 8, 6).astype(np.float64)
        t = t[t[:, 0, 0] > 0]
        tot = t[:, :, 0].mean()
        clk = (t[:, :, 0] / (t[:, :, 5] / 100.0)).mean() / 1e3
        print(f"   trace ({len(t)} blocks, clock {clk:.2f} GHz): total {tot:.0f} cyc; issue "
              f"{t[:, :, 1].mean() / tot:.3f} kloop {t[:, :, 2].mean() / tot:.3f} barrier "
              f"{t[:, :, 3].mean() / tot:.3f} epilogue {t[:, :, 4].mean() / tot:.3f}; per-wave barrier "
              + " ".join(f"{v:.2f}" for v in (t[:, :, 3].mean(0) / tot)))
    peak = 2516.6 / {2: 3, 3: 6, 16: 3}[pieces]
    tf = flops / us / 1e6
    print(f"{name:12s} {kind:5s} {cin:3d}->{cout:3d} @{H:3d}  {us:8.1f} us  {tf:6.1f} TF/s  "
          f"{tf / peak:5.3f} of peak", flush=True)
    return us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--pieces", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--only", default="")
    ap.add_argument("--warm", type=float, default=1.0, help="seconds of untimed launches first")
    a = ap.parse_args()
    names = [n for n in CASES if not a.only or n in a.only.split(",")]
    for n in names:
        run(n, a.reps, a.pieces, a.batch, a.warm)


if __name__ == "__main__":
    main()
