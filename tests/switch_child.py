"""Child process of tests/test_gpu_switches.py: the benchmarked forward_backward under the
EBSDVAE_* library switch set in this process's environment (libebsdvae.so reads those once,
at first use), checked against the pinned oracle exactly like tests/test_gpu_fullsize.py.

    python tests/switch_child.py PRECISIONS COPIES     (e.g. "f16x3,bf16x6" 1)
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "ebsd-vae_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pinned import check_grads, fixture  # noqa: E402
from latice import _native, engine as E  # noqa: E402
from latice.model import VariationalAutoEncoderRawData  # noqa: E402
from latice.trainer import VAETrainer  # noqa: E402


def main():
    precs, copies = sys.argv[1].split(","), int(sys.argv[2])
    _native.load()
    dev = torch.device("cuda:0")
    name = "vae128_b4"
    f, sd = fixture(name)
    b = int(f["meta"][0])
    m = VariationalAutoEncoderRawData(32, int(f["meta"][2]), int(f["meta"][1]))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.to(dev)
    x = torch.from_numpy(np.ascontiguousarray(np.tile(f["x"], (copies, 1, 1, 1)))).to(dev)
    eps = torch.from_numpy(np.ascontiguousarray(np.tile(f["eps"], (copies, 1)))).to(dev)
    for prec in precs:
        with E.precision(prec):
            tr = VAETrainer(m, kl_lambda=float(f["kl_lambda"]))
            with E.record_state() as rec:
                loss, _, _ = tr.forward_backward(x, eps)
            torch.cuda.synchronize()
        err = abs(float(loss) - float(f["loss"])) / abs(float(f["loss"]))
        assert err <= 1e-5, f"{prec}: loss rel err {err:.2e}"
        rec0 = {n: (y[:b], st[:b]) for n, (y, st) in rec.items()}
        switches = {k: v for k, v in os.environ.items() if k.startswith("EBSDVAE_")}
        check_grads(name, m.plan, rec0, tr.G, label=f"{switches} {prec} B={b * copies}", prec=prec)
    print("switch child OK")


if __name__ == "__main__":
    main()
