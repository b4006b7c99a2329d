"""Time PackSet.refresh() (the per-step weight packing: pack_wmax_kernel + pack_split_kernel)
for the c2 model at B = 256:  python tools/pack_micro.py [--reps 200]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ebsd-vae_amd")]

import torch  # noqa: E402

from latice import engine as E  # noqa: E402
from latice.model import VariationalAutoEncoderRawData  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    m = VariationalAutoEncoderRawData(32, 16, 128).cuda()
    params = dict(m.named_parameters())
    ps = E.PackSet(m.plan, params)
    for _ in range(10):
        ps.refresh()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s = torch.cuda.current_stream()
    e0.record(s)
    for _ in range(a.reps):
        ps.refresh()
    e1.record(s)
    torch.cuda.synchronize()
    print(f"PackSet.refresh: {e0.elapsed_time(e1) * 1000 / a.reps:.1f} us per call "
          f"({sum(n for _, _, n in ps.batches)} packs)")


if __name__ == "__main__":
    main()
