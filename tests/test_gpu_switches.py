"""Every EBSDVAE_* environment switch that still selects other device code or another schedule,
on the benchmarked path (VAETrainer.forward_backward) -- so no alternative stays linked
without a test:

  * schedule switches (where the work runs and which events order it -- the weight-gradient
    side stream, kernel-attached forks, light event waits, side-stream work inside a captured
    graph): the gradient must be BITWISE equal to the default run's.  Every reduction has a
    fixed order, so a difference can only be an ordering bug, e.g. a weight gradient that read
    gy before the apply wrote it (EBSDVAE_KFORK);
  * arithmetic switches (another kernel or fusion for the same math): the pinned-oracle gates
    of tests/pinned.py, as in test_gpu_trainer.py.

Switches the Python layer reads at call time are flipped in-process; those libebsdvae.so reads
once (conv / weight-gradient planners) run in a child process each (tests/switch_child.py).
Build / tooling variables (EBSDVAE_LIB, EBSDVAE_ARCH, EBSDVAE_PRECISION -- covered by the
precision parametrisations -- and EBSDVAE_BENCH_LAUNCHER) select no alternative kernel.
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from pinned import check_grads, fixture
from latice import engine as E
from latice import model as M
from latice.model import VariationalAutoEncoderRawData
from latice.trainer import VAETrainer

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _model(device, name="vae128_b4"):
    f, sd = fixture(name)
    m = VariationalAutoEncoderRawData(32, int(f["meta"][2]), int(f["meta"][1]))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return f, m.to(device)


def _grad(m, f, device, copies=1):
    x = torch.from_numpy(np.ascontiguousarray(np.tile(f["x"], (copies, 1, 1, 1)))).to(device)
    eps = torch.from_numpy(np.ascontiguousarray(np.tile(f["eps"], (copies, 1)))).to(device)
    tr = VAETrainer(m, kl_lambda=float(f["kl_lambda"]))
    with E.record_state() as rec:
        tr.forward_backward(x, eps)
    torch.cuda.synchronize()
    return tr, rec


@pytest.mark.parametrize("attr", ["_KFORK", "_LIGHT_EVENTS", "_WG_STREAM", "_ON_MAIN_FINAL"])
@pytest.mark.parametrize("copies", [1, 64], ids=["B4", "B256"])
def test_schedule_switch_gives_bitwise_equal_gradients(cuda, monkeypatch, attr, copies):
    """EBSDVAE_KFORK=0 / EBSDVAE_LIGHT_EVENTS=0 / EBSDVAE_WGRAD_STREAM=0 /
    EBSDVAE_FINAL_REDUCE_SIDE=1 against the default."""
    f, m = _model(cuda)
    tr0, _ = _grad(m, f, cuda, copies)
    g0 = tr0.gflat.clone()
    monkeypatch.setattr(E, attr, False)
    tr1, _ = _grad(m, f, cuda, copies)
    assert torch.equal(tr1.gflat, g0), f"{attr}=0 changed the gradient"


def test_graph_side_switch_gives_bitwise_equal_steps(cuda, monkeypatch):
    """EBSDVAE_GRAPH_SIDE=0 (captured step keeps everything on one stream): the same
    parameters after capture + one replay (two Adam steps) as with the side stream inside
    the graph."""
    f, _ = _model(cuda)
    x = torch.from_numpy(np.ascontiguousarray(np.tile(f["x"], (16, 1, 1, 1)))).to(cuda)
    flats = []
    for side in (True, False):
        _, m = _model(cuda)
        monkeypatch.setattr(E, "_GRAPH_SIDE", side)
        tr = VAETrainer(m, kl_lambda=float(f["kl_lambda"]), seed=5)
        tr.capture(x, warmup=1)
        tr.replay()
        torch.cuda.synchronize()
        flats.append(tr.flat.clone())
    assert torch.equal(flats[0], flats[1])


@pytest.mark.parametrize("switch", ["attr:_FIRST_VALU", "attr:_NET_END", "env:EBSDVAE_POOL_OUT",
                                    "env:EBSDVAE_WGRAD_F16", "env:EBSDVAE_POOL_REDUCE",
                                    "env:EBSDVAE_UPSUM", "on:_DWFUSE"])
@pytest.mark.parametrize("prec", ["f16x3", "bf16x6"])
def test_arithmetic_switch_meets_pinned_gates(cuda, monkeypatch, switch, prec):
    kind, name = switch.split(":")
    if kind == "attr":
        monkeypatch.setattr(E, name, False)
    elif kind == "on":   # an opt-in path (EBSDVAE_DWFUSE=1: the fused input + weight gradient)
        monkeypatch.setattr(E, name, True)
    else:
        monkeypatch.setenv(name, "0")
    f, m = _model(cuda)
    with E.precision(prec):
        tr, rec = _grad(m, f, cuda)
    check_grads("vae128_b4", m.plan, rec, tr.G, label=f"{name}=0 {prec}", prec=prec)


def test_inference_switches_keep_outputs(cuda, monkeypatch):
    """EBSDVAE_EVAL_Y=1 (pooled producers also write y in inference) and
    EBSDVAE_DEFER_DECODE=0 (x_hat computed at model(x)): bitwise the default outputs.  The
    first block's statistics from its fma chain (EBSDVAE_FIRST_GRAM=0) in both: with the
    deferral off the call takes the training-mode encoder, whose statistics are the fp32
    two-pass ones, not the inference path's moment-based ones."""
    monkeypatch.setattr(E, "_FIRST_GRAM", False)
    f, m = _model(cuda)
    m.eval()
    x = torch.from_numpy(f["x"]).to(cuda)
    eps = torch.from_numpy(f["eps"]).to(cuda)

    def run():
        with torch.no_grad():
            z, xh, mu, std = m(x, eps=eps)
            return [t.clone() for t in (z, xh * 1.0, mu, std)]
    ref = run()
    monkeypatch.setattr(E, "_EVAL_Y", True)
    assert all(torch.equal(a, b) for a, b in zip(run(), ref))
    monkeypatch.setattr(E, "_EVAL_Y", False)
    monkeypatch.setattr(M, "_DEFER", False)
    out = run()
    assert all(torch.equal(a, b) for a, b in zip(out, ref))


# library-level switches: (variable, value, precisions, copies).  Copies = 64 (B = 256) where
# the switch only matters at the full batch (in-kernel finalize, weight-gradient block target)
LIB_SWITCHES = [
    ("EBSDVAE_CONV_PIPE", "0", "f16x3,bf16x6", 1),
    ("EBSDVAE_CONV_SMALL1", "0", "f16x3", 1),
    ("EBSDVAE_CONV_MULTI_IMAGE", "0", "f16x3,bf16x6", 1),
    ("EBSDVAE_WRES", "0", "f16x3", 1),
    ("EBSDVAE_FUSE_FINALIZE", "0", "f16x3", 64),
    ("EBSDVAE_WG_PIPE", "0", "f16x3,bf16x6", 1),
    ("EBSDVAE_WG_CO128", "0", "f16x3", 1),
    ("EBSDVAE_WG_TW", "32", "bf16x6", 1),
    ("EBSDVAE_WG_BLOCKS", "1024", "f16x3", 64),
    ("EBSDVAE_FORK_DEVICE_SCOPE", "1", "f16x3", 1),   # round 6: device-scope fork events (A/B)
]


@pytest.mark.parametrize("var,val,precs,copies", LIB_SWITCHES, ids=[s[0][8:] for s in LIB_SWITCHES])
def test_library_switch_meets_pinned_gates(cuda, var, val, precs, copies):
    env = dict(os.environ, **{var: val})
    r = subprocess.run([sys.executable, os.path.join(HERE, "switch_child.py"), precs, str(copies)],
                       env=env, capture_output=True, text=True, timeout=110)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stderr[-3000:]
    assert "switch child OK" in r.stdout
