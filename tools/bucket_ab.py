"""A/B of the trainer's bucket layout on one GPU: a world-1 `nccl` group with the all-reduces
forced on (GradReducer(force=True)), so the step issues every bucket's collective exactly as
at N > 1 (world 1: RCCL's copy kernels only).  Variants: three buckets (bucket 1 started after
the deep encoder layers' weight gradients, their slice reductions flushed early) and two
buckets (the round-4 layout: decoder + heads, then the whole encoder after the backward), and
no collective at all (the reducer inactive, as at N = 1).

    python tools/bucket_ab.py [--steps 20] [--rounds 3]
    GPU_MAX_HW_QUEUES=8 python tools/bucket_ab.py    # what bench.py and latice set (this script
                                                     # initialises HIP before importing latice: 4)
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ebsd-vae_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from latice.model import VariationalAutoEncoderRawData
    from latice.seeding import seeded_state_dict, synthetic_patterns
    from latice.trainer import GradReducer, VAETrainer
    model = VariationalAutoEncoderRawData()
    model.load_state_dict({k: torch.from_numpy(v) for k, v in seeded_state_dict(0).items()})
    model = model.to(dev)
    tr = VAETrainer(model, force_allreduce=True)
    x = torch.from_numpy(synthetic_patterns(0, 256, 128)).to(dev)
    three = (tr._deep_last, tr.reducer)
    two = (None, GradReducer(tr.gflat, tr.split, force=True))
    none = (None, GradReducer(tr.gflat, tr.split))   # world 1, not forced: no collective

    def timed(cfg):
        tr._deep_last, tr.reducer = cfg
        for _ in range(3):
            tr.step(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            tr.step(x)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.steps * 1e3

    for r in range(args.rounds):
        a, b, c = timed(three), timed(two), timed(none)
        print(f"round {r}: three buckets {a:.3f} ms/step, two buckets {b:.3f}, no collective "
              f"{c:.3f}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
