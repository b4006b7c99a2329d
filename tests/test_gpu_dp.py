"""Data-parallel equivalence of the benchmarked trainer on the GPU: two ranks (separate
processes, torch.distributed gloo, both on cuda:0) each run VAETrainer.forward_backward on
their half of a batch -- the loss kernel's gradient pre-scaled by 1/W, the two-bucket
all-reduce -- and must hold the single-process gradient of the whole batch.  Rank 1 starts
from different weights, so the init broadcast is checked too.
The RCCL ("nccl") path differs only in the backend string; it is exercised by the driver's
multi-GPU bench."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from latice.model import VariationalAutoEncoderRawData
from latice.seeding import seeded_eps, seeded_state_dict, synthetic_patterns
from latice.trainer import VAETrainer

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("prec", ["f16x3", "fp32"])
def test_two_rank_gradient_equals_single_process(cuda, tmp_path, prec):
    world, port = 2, _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), DP_OUT=str(tmp_path), DP_PREC=prec)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dp_trainer_worker.py")],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = [p.communicate(timeout=150)[0].decode() for p in procs]
    for p, out in zip(procs, outs):   # the tail of a failing worker's output, untruncated
        if p.returncode != 0:
            print(out[-6000:])
    assert all(p.returncode == 0 for p in procs), [o[-300:] for o in outs]
    from latice import engine as E
    with E.precision(prec):
        m = VariationalAutoEncoderRawData()
        m.load_state_dict({k: torch.from_numpy(v) for k, v in seeded_state_dict(0).items()})
        tr = VAETrainer(m.to(cuda), kl_lambda=5e-6)
        x = torch.from_numpy(synthetic_patterns(9, 4 * world)).to(cuda)
        eps = torch.from_numpy(seeded_eps(9, 4 * world)).to(cuda)
        loss, _, _ = tr.forward_backward(x, eps)
        g = tr.gflat.cpu().numpy().astype(np.float64)
    flat = [np.load(tmp_path / f"flat{r}.npy") for r in range(world)]
    assert np.array_equal(flat[0], flat[1])                       # broadcast at init
    assert np.array_equal(flat[0], tr.flat.cpu().numpy())
    for r in range(world):
        gr = np.load(tmp_path / f"gflat{r}.npy").astype(np.float64)
        err = np.abs(gr - g).max() / np.abs(g).max()
        print(f"\nrank {r} all-reduced gradient vs single process 2B: {err:.2e}")
        assert err < 1e-5
    losses = [float(np.load(tmp_path / f"loss{r}.npy")[0]) for r in range(world)]
    assert abs(np.mean(losses) - float(loss)) < 1e-6 * abs(float(loss))


def test_nccl_side_stream_allreduce_world1(cuda):
    """The RCCL path of the benchmarked step, executed: an "nccl" process group of one rank
    with the trainer's GradReducer forced active, so bucket 0 is all-reduced from the
    weight-gradient side stream (behind the heads backward) and bucket 1 after the join, and
    finish() orders both before Adam.  A SUM over one rank is the identity, so the flat
    gradient and the parameters after the step must be bitwise those of the non-DP step."""
    import datetime
    import torch.distributed as dist
    from latice import engine as E
    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                            device_id=cuda, timeout=datetime.timedelta(seconds=120))
    try:
        assert dist.get_backend() == "nccl"
        sd = {k: torch.from_numpy(v) for k, v in seeded_state_dict(0).items()}
        x = torch.from_numpy(synthetic_patterns(3, 8)).to(cuda)
        eps = torch.from_numpy(seeded_eps(3, 8)).to(cuda)
        out = {}
        for tag, force in (("plain", False), ("rccl", True)):
            m = VariationalAutoEncoderRawData()
            m.load_state_dict(sd)
            tr = VAETrainer(m.to(cuda), kl_lambda=5e-6, force_allreduce=force)
            assert tr.reducer.active == force and tr.world == 1
            assert E.side_streams_enabled()
            tr.time_allreduce = True
            tr.forward_backward(x, eps)
            exposed = tr.allreduce_exposed_ms()   # bench.py's allreduce_exposed_ms
            assert (exposed is None) == (not force)
            if force:
                assert 0.0 <= exposed < 1e3
            g = tr.gflat.clone()
            tr.optimizer_step()
            torch.cuda.synchronize()
            out[tag] = (g.cpu(), tr.flat.clone().cpu())
        assert torch.equal(out["plain"][0], out["rccl"][0])
        assert torch.equal(out["plain"][1], out["rccl"][1])
        # and a real collective on the device: the bench's float64 MAX all-reduce
        t = torch.tensor([1.5, -2.0], device=cuda, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        assert t.tolist() == [1.5, -2.0]
    finally:
        dist.destroy_process_group()


def test_bench_self_launches_ranks(cuda):
    """`python bench.py --gpus 2` with no launcher spawns two ranks itself (the driver may run
    it that way); here gloo, both ranks on this one GPU.  The line must report the group that
    actually formed."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(HERE), "bench.py"), "--gpus", "2",
                        "--steps", "2", "--warmup", "1", "--batch", "8", "--dist-backend", "gloo",
                        "--no-cpu-baseline", "--strict-fp32-steps", "0", "--c4-batches", "0",
                        "--c5-steps", "0", "--no-probe"],
                       env=env, capture_output=True, timeout=240, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["global_batch"] == 16
    assert res["process_group"]["backend"] == "gloo" and res["process_group"]["world_size"] == 2
    assert len(res["rank_ms_per_step"]) == 2 and res["rank_spread_pct"] >= 0
    assert res["allreduce_exposed_ms"] is not None and res["allreduce_exposed_ms"] >= 0
    assert "gloo grad all-reduce (rehearsal" in res["config"]["workload"]
