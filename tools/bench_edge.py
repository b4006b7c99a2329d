"""Micro-timing of the final conv(32->1) forward vs a plain streaming read of its input."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ebsd-vae_amd")]
import torch  # noqa: E402

from latice import _native as N  # noqa: E402
from latice import engine as E  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


B, S, C = 256, 128, 32
y = torch.randn(B, S, S, C, device="cuda")
st = torch.stack([torch.zeros(B, C), torch.ones(B, C)], -1).cuda().contiguous()
w = torch.randn(1, C, 3, 3, device="cuda") * 0.1
b = torch.zeros(1, device="cuda")
out = torch.empty(B, 1, S, S, device="cuda")
us = timeit(lambda: N.call("ebsdvae_conv3x3_cout1_fwd", N.ptr(y), N.ptr(st), E.ACT_NORM, N.ptr(w),
                           N.ptr(b), N.ptr(out), 0, B, S, S, C, N.stream()))
print(f"cout1_fwd NORM  {us:8.1f} us  {y.numel() * 4 / us / 1e3:7.1f} GB/s of input")
us = timeit(lambda: N.call("ebsdvae_conv3x3_cout1_fwd", N.ptr(y), None, E.ACT_RAW, N.ptr(w),
                           None, N.ptr(out), 1, B, S, S, C, N.stream()))
print(f"cout1_fwd RAW   {us:8.1f} us")
z = torch.empty_like(y)
us = timeit(lambda: z.copy_(y))
print(f"torch copy      {us:8.1f} us  {2 * y.numel() * 4 / us / 1e3:7.1f} GB/s")
