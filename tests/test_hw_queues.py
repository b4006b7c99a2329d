"""`import latice` defaults GPU_MAX_HW_QUEUES to 8 before HIP initialises,
keeps a value the user set, and warns when HIP was initialised first, since the variable can no
longer take effect then.  Each case imports latice in a fresh interpreter;
HIP initialisation is simulated (no GPU is touched)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "ebsd-vae_amd")

CHILD = r"""
import os, sys, warnings
sys.path.insert(0, {pkg!r})
import torch
if {late}:
    torch.cuda.is_initialized = lambda: True   # as if a HIP call had happened already
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter("always")
    import latice
print("QUEUES", os.environ.get("GPU_MAX_HW_QUEUES"))
print("WARNED", any(issubclass(x.category, RuntimeWarning) and "GPU_MAX_HW_QUEUES" in str(x.message) for x in w))
"""


def _run(late, preset=None):
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    if preset is not None:
        env["GPU_MAX_HW_QUEUES"] = preset
    r = subprocess.run([sys.executable, "-c", CHILD.format(pkg=PKG, late=late)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = dict(line.split(" ", 1) for line in r.stdout.splitlines() if line.startswith(("QUEUES", "WARNED")))
    return out["QUEUES"], out["WARNED"] == "True"


def test_default_set_before_hip():
    assert _run(late=False) == ("8", False)


def test_user_value_kept():
    assert _run(late=False, preset="12") == ("12", False)


def test_warns_when_hip_initialised_first():
    assert _run(late=True) == ("8", True)


def test_no_warning_when_user_set_it():
    assert _run(late=True, preset="8") == ("8", False)
