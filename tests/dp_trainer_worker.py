"""Worker of tests/test_gpu_dp.py (not a test module): one data-parallel rank of
VAETrainer on cuda:0 over torch.distributed gloo.  Env: RANK, WORLD_SIZE, MASTER_ADDR,
MASTER_PORT, DP_OUT (output directory), DP_PREC (conv arithmetic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "ebsd-vae_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from latice import engine as E
    from latice.model import VariationalAutoEncoderRawData
    from latice.seeding import seeded_eps, seeded_state_dict, synthetic_patterns
    from latice.trainer import VAETrainer, shard_batch
    E.set_precision(os.environ.get("DP_PREC", "f16x3"))
    dev = torch.device("cuda:0")
    # rank r > 0 starts from DIFFERENT weights: VAETrainer must broadcast rank 0's
    m = VariationalAutoEncoderRawData()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in seeded_state_dict(rank * 17).items()})
    m = m.to(dev)
    tr = VAETrainer(m, kl_lambda=5e-6, seed=100 + rank)
    x = shard_batch(torch.from_numpy(synthetic_patterns(9, 4 * world)), rank, world).to(dev)
    eps = shard_batch(torch.from_numpy(seeded_eps(9, 4 * world)), rank, world).to(dev)
    loss, _, _ = tr.forward_backward(x, eps)
    torch.cuda.synchronize()
    out = os.environ["DP_OUT"]
    np.save(os.path.join(out, f"flat{rank}.npy"), tr.flat.cpu().numpy())
    np.save(os.path.join(out, f"gflat{rank}.npy"), tr.gflat.cpu().numpy())
    np.save(os.path.join(out, f"loss{rank}.npy"), np.array([float(loss)]))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
