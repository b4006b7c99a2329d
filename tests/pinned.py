"""Shared gradient check of the GPU backward against the decision- and state-pinned float64
oracle (oracle/vae_oracle.py: pinned_routing, forward_from_state).

Two comparisons per parameter gradient g (norm-wise max|d|/max|ref|):
  decision-pinned  the float64 oracle's own forward, with only the discrete routing --
                   max-pool argmax and LeakyReLU branch of every block -- taken from the GPU
                   run (the same rule the HIP backward applies to its saved y).  End-to-end
                   float64 agreement: gate 1e-3 on every fixture.
  state-pinned     the float64 backward evaluated on the GPU run's own forward state (its
                   saved pre-norm y and InstanceNorm {mean, rstd} of every block) and
                   routing: isolates the backward arithmetic, gate 1e-4.  This matters on
                   vae128_b2_edge, whose constant (saturated) pattern makes the first
                   InstanceNorm run over a near-constant plane (rstd ~ 1e2): there any
                   float32 forward is far more sensitive (numpy's own float32 run lands
                   4e-2 from float64 with identical routing; the HIP run 2e-4).
Measured on MI355X (round 2): decision-pinned <= 2.2e-4, state-pinned <= 3.4e-5 over all
fixtures and the fp32 / bf16x6 / f16x3 arithmetics.
The 19 conv biases feeding an affine-free InstanceNorm have an analytically zero gradient
(sum_{b,h,w} gy = 0): what an fp32 run returns is the rounding residue of that cancellation,
which scales with the magnitude of the summed terms, A_c = sum_{b,h,w} |gy| (the oracle's,
vae_oracle.backward(absum=...)), not with the batch.  Gate: |g_c| <= ZERO_BIAS_K * 2^-24 * A_c
per channel (the reference's own fp32 residue at B=256 is recorded in
tests/golden/bias_noise_b256.npz by make_bias_noise.py).
"""
import functools
import os

import numpy as np

from conftest import GOLDEN
from latice.seeding import seeded_state_dict
from oracle import vae_oracle as O

ZERO_GRAD_BIAS = tuple(f"encoder.{i}.0.bias" for i in O.ENC_IDX) + tuple(
    f"decoder.{i}.0.bias" for i in O.DEC_IDX)
DECISION_GATE = 1e-3
STATE_GATE = 1e-4
# residue gate, in units of 2^-24 * A_c, per conv arithmetic (the one in effect when check_grads
# runs).  Measured on MI355X (round 4, every fixture, B = 4..256, every switch): f16x3 <= 3.0,
# bf16x6 <= 1.7, fp32 <= 1.4.  Round 6's MFMA network end forms the last block's reduce sums
# from a two-piece fp16 g1: <= 1.1 on the well-conditioned fixtures, 4.3 / 6.5 / 3.6 (f16x3 /
# bf16x6 / fp32) on the saturated vae128_b2_edge, on decoder.13.0.  One fp32 run (round 5,
# gpurun_out/t_sw1.txt) returned 180.8 on decoder.13.0 with a 200x weight-gradient error on the
# same layer while the layers whose gradients flow through decoder.13's gy were exact: most
# likely decoder.13's side-stream weight gradient read a gy13 that differed from the one the
# main stream's input gradient read; the cause is not established.  No
# run since has repeated it; the poison-mode suite (tests/test_gpu_poison.py, and every repeat
# of tests/test_gpu_determinism.py) turns such a read into NaN instead of an in-tolerance error.
# The reference's own fp32 run at B = 256: 0.18 (bias_noise_b256.npz).
ZERO_BIAS_K = {"f16x3": 16.0, "bf16x6": 16.0, "bf16x3": 16.0, "fp32": 16.0}
U32 = 2.0 ** -24


@functools.lru_cache(maxsize=4)
def fixture(name):
    f = O.load_fixture(os.path.join(GOLDEN, name + ".npz"))
    B, S, L, ws, xs = (int(v) for v in f["meta"])
    sd = seeded_state_dict(ws, 32, L, S)
    return f, sd


@functools.lru_cache(maxsize=4)
def oracle_fp64(name):
    f, sd = fixture(name)
    outs, cache = O.forward(sd, f["x"], f["eps"])
    return outs, cache


def host(t):
    return t.detach().double().cpu().numpy()


def blocks(plan, rec):
    """(enc_blocks, dec_blocks) [(y, st)] of a recorded GPU forward (engine.record_state)."""
    def one(L):
        y, st = rec[L.name]
        return y.detach().float().cpu().numpy(), st.detach().float().cpu().numpy()
    return [one(L) for L in plan.enc], [one(L) for L in plan.dec]


def check_grads(name, plan, rec, grads, label="", prec=None):
    """grads: {state_dict name: GPU gradient tensor}; prec: the conv arithmetic that computed
    them (default: the one in effect now).  Prints every error, then asserts."""
    from latice import engine as E
    prec = prec or E.get_precision()
    kz = ZERO_BIAS_K[prec]
    f, sd = fixture(name)
    kl = float(f["kl_lambda"])
    enc_b, dec_b = blocks(plan, rec)
    _, cache_s, pins = O.forward_from_state(sd, f["x"], f["eps"], enc_b, dec_b)
    g_state = O.backward(cache_s, f["x"], kl, pins=pins)
    _, cache64 = oracle_fp64(name)
    absum = {}
    g_dec = O.backward(cache64, f["x"], kl, pins=pins, absum=absum)
    rows, fails = [], []
    for n in g_state:
        g = host(grads[n])
        if n in ZERO_GRAD_BIAS:
            # residue in units of 2^-24 * A_c, worst channel
            a = float((np.abs(g) / (U32 * np.maximum(absum[n], 1e-300))).max())
            rows.append((n, a, None))
            if a > kz:
                fails.append((n, "zero-bias", a))
            continue
        es, ed = O.rel_err(g, g_state[n]), O.rel_err(g, g_dec[n])
        rows.append((n, es, ed))
        if es > STATE_GATE:
            fails.append((n, "state", es))
        if ed > DECISION_GATE:
            fails.append((n, "decision", ed))
    worst_s = max(r[1] for r in rows if r[2] is not None)
    worst_d = max(r[2] for r in rows if r[2] is not None)
    worst_b = max(r[1] for r in rows if r[2] is None)
    print(f"\n[{label} {name}] worst weight-grad err: state-pinned {worst_s:.2e}, "
          f"decision-pinned {worst_d:.2e}; worst zero-grad bias residue {worst_b:.1f} x 2^-24 A "
          f"(gate {kz:g}, {prec})")
    for n, a, b in rows:
        print(f"    {n:22s} " + (f"residue {a:.1f} x 2^-24 A" if b is None else f"state {a:.2e}  decision {b:.2e}"))
    assert not fails, fails
    return worst_s, worst_d
