"""A/B of eager step() vs hipGraph replay of the whole training step (N = 1)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ebsd-vae_amd")]
import torch  # noqa: E402

from latice.model import VariationalAutoEncoderRawData  # noqa: E402
from latice.seeding import seeded_state_dict, synthetic_patterns  # noqa: E402
from latice.trainer import VAETrainer  # noqa: E402


def timeit(fn, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


m = VariationalAutoEncoderRawData()
m.load_state_dict({k: torch.from_numpy(v) for k, v in seeded_state_dict(0).items()})
m = m.cuda()
tr = VAETrainer(m)
x = torch.from_numpy(synthetic_patterns(0, 256)).cuda()
for _ in range(5):
    tr.step(x)
e = timeit(lambda: tr.step(x), 20)
tr.capture(x)
g = timeit(tr.replay, 20)
e2 = timeit(lambda: tr.step(x), 20)
g2 = timeit(tr.replay, 20)
print(f"eager {e:.3f} / {e2:.3f} ms   graph {g:.3f} / {g2:.3f} ms")
# CPU-side enqueue time of one eager step (no synchronisation inside the measured loop)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    tr.step(x)
cpu = (time.perf_counter() - t0) / 10 * 1e3
torch.cuda.synchronize()
print(f"eager CPU enqueue {cpu:.3f} ms/step")
