"""Stand-alone timing of the HBM-bound network-end kernels at B=256, 128x128 (the first conv
1->32, the final conv 32->1, the fused InstanceNorm-backward passes of the two 32-channel
end blocks, and the generic InstanceNorm-backward apply), as GB/s of algorithmic bytes.

    python tools/edge_micro.py [--reps 20] [--only small1,cout1,...]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ebsd-vae_amd")]

import torch  # noqa: E402

from latice import _native as N  # noqa: E402
from latice.engine import ACT_NORM, ACT_RAW, P_ID  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = torch.device("cuda")
    B, H, C = a.batch, 128, 32
    g = torch.Generator(device=dev).manual_seed(0)
    s = N.stream()
    x = torch.rand(B, H, H, 1, device=dev, generator=g)
    y = torch.randn(B, H, H, C, device=dev, generator=g)
    y2 = torch.randn(B, H, H, C, device=dev, generator=g)
    gy = torch.empty(B, H, H, C, device=dev)
    st = torch.stack([torch.zeros(B, C, device=dev), torch.ones(B, C, device=dev)], -1).contiguous()
    bst = torch.zeros(B, C, 2, device=dev)
    w1 = torch.randn(8 * 10 * C, device=dev, generator=g) * 0.1   # packed first-conv weight (timing only)
    w14 = torch.randn(1, C, 3, 3, device=dev, generator=g) * 0.1
    b = torch.zeros(C, device=dev)
    g1 = torch.randn(B, H, H, 1, device=dev, generator=g)
    out1 = torch.empty(B, H, H, 1, device=dev)
    T = N.call("ebsdvae_in_bwd_tiles", H, H, C)
    part = torch.empty(B, T, C, 2, dtype=torch.float64, device=dev)
    wpart = torch.empty(B * T, 9, C, device=dev)
    bpart = torch.empty(B * T * C, device=dev)
    yc = torch.empty(B, H, H, C, device=dev)
    spart = torch.empty(B, N.call("ebsdvae_conv3x3_stat_tiles", H, H, C), C, 2, device=dev)
    E4 = B * H * H * C * 4
    Tn = N.call("ebsdvae_net_end_tiles", H, H)
    ne_out = [torch.empty(B, H, H, device=dev) for _ in range(2)]
    ne_bce = torch.empty(B, max(Tn, 1), device=dev)
    ne_part = torch.empty(B, max(Tn, 1), C, 2, dtype=torch.float64, device=dev)
    ne_w = torch.empty(B * max(Tn, 1), 9, C, device=dev)
    ne_b = torch.empty(B * max(Tn, 1), device=dev)
    one = torch.ones((), device=dev)
    w0 = torch.randn(C, 1, 3, 3, device=dev, generator=g) * 0.3
    Tf = N.call("ebsdvae_conv_first_stat_tiles", H, H)
    fpart = torch.empty(B, Tf, C, 2, device=dev)
    cases = {
        "first_valu": (lambda: N.call("ebsdvae_conv_first_fwd", N.ptr(x), N.ptr(w0), N.ptr(b), N.ptr(yc),
                                      N.ptr(fpart), B, H, H, C, s), E4 + E4 // 32),
        # inference's first-conv statistics from the moments of x (reads x only)
        "first_stats": (lambda: N.call("ebsdvae_conv_first_stats", N.ptr(x), N.ptr(w0), N.ptr(b),
                                       N.ptr(fpart), B, H, H, C, s), E4 // 32),
        "first_rc": (lambda: N.call("ebsdvae_in_bwd_first_apply_wgrad_rc", N.ptr(y2), N.ptr(w0), N.ptr(b),
                                    N.ptr(st), N.ptr(bst), N.ptr(x), N.ptr(wpart), N.ptr(bpart),
                                    B, H, H, C, s), E4 + E4 // 32),
        "net_end": (lambda: N.call("ebsdvae_net_end", N.ptr(y), N.ptr(st), N.ptr(w14), N.ptr(b), N.ptr(x),
                                   N.ptr(one), 1.0, N.ptr(ne_out[0]), N.ptr(ne_out[1]), N.ptr(ne_bce),
                                   ne_part.data_ptr(), N.ptr(ne_w), N.ptr(ne_b), B, H, H, C, s),
                    E4 + 3 * E4 // 32),
        "net_end_valu": (lambda: N.call("ebsdvae_net_end_valu", N.ptr(y), N.ptr(st), N.ptr(w14), N.ptr(b),
                                        N.ptr(x), N.ptr(one), 1.0, N.ptr(ne_out[0]), N.ptr(ne_out[1]),
                                        N.ptr(ne_bce), ne_part.data_ptr(), N.ptr(ne_w), N.ptr(ne_b), B, H, H,
                                        C, s),
                         E4 + 3 * E4 // 32),
        # name: (launch, algorithmic bytes)
        "small1": (lambda: N.call("ebsdvae_conv3x3_fwd", N.ptr(x), None, ACT_RAW, N.ptr(w1), N.ptr(b),
                                  N.ptr(yc), N.ptr(spart), None, B, H, H, 1, C, s), E4 + E4 // 32),
        "cout1": (lambda: N.call("ebsdvae_conv3x3_cout1_fwd", N.ptr(y), N.ptr(st), ACT_NORM, N.ptr(w14),
                                 N.ptr(b), N.ptr(out1), 0, B, H, H, C, s), E4 + E4 // 32),
        "final_reduce": (lambda: N.call("ebsdvae_in_bwd_final_reduce", N.ptr(g1), N.ptr(w14), N.ptr(y),
                                        N.ptr(st), part.data_ptr(), N.ptr(wpart), N.ptr(bpart),
                                        B, H, H, C, s), E4 + E4 // 32),
        "final_apply": (lambda: N.call("ebsdvae_in_bwd_final_apply", N.ptr(g1), N.ptr(w14), N.ptr(y),
                                       N.ptr(st), N.ptr(bst), N.ptr(gy), B, H, H, C, s), 2 * E4 + E4 // 32),
        "first_apply": (lambda: N.call("ebsdvae_in_bwd_first_apply_wgrad", N.ptr(y2), N.ptr(y), N.ptr(st),
                                       N.ptr(bst), N.ptr(x), N.ptr(wpart), N.ptr(bpart), B, H, H, C, s),
                        2 * E4 + E4 // 32),
        # references: torch's own streaming kernels on the same tensors
        "ref_fill": (lambda: yc.fill_(1.0), E4),
        "ref_copy": (lambda: yc.copy_(y), 2 * E4),
        "ref_sum": (lambda: torch.sum(y, dim=(1, 2)), E4),
        "in_apply": (lambda: N.call("ebsdvae_in_bwd_apply", N.ptr(y2), P_ID, N.ptr(y), N.ptr(st),
                                    N.ptr(bst), N.ptr(gy), B, H, H, C, s), 3 * E4),
    }
    names = [n for n in cases if not a.only or n in a.only.split(",")]
    for n in names:
        fn, nbytes = cases[n]
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t_end = time.time() + 0.5
        while time.time() < t_end:
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        print(f"{n:13s} {us:8.1f} us  {nbytes / us / 1e3:7.0f} GB/s  ({nbytes / 1e6:.0f} MB)", flush=True)


if __name__ == "__main__":
    main()
