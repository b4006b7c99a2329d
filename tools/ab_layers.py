"""Same-box A/B of per-layer conv timings across library builds.

    python tools/ab_layers.py base=ebsd-vae_amd/lib/libebsdvae.so exp=ebsd-vae_amd/lib/libebsdvae_x.so \
        knob=ebsd-vae_amd/lib/libebsdvae.so:EBSDVAE_CONV32=1

Runs tools/layer_profile.py once per library (EBSDVAE_LIB=...) in child processes and
prints one table with a ms/step column per build.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(spec):
    """spec = lib[:VAR=VAL[,VAR=VAL...]]"""
    lib, _, envs = spec.partition(":")
    env = dict(os.environ, EBSDVAE_LIB=os.path.join(ROOT, lib))
    for kv in filter(None, envs.split(",")):
        k, v = kv.split("=", 1)
        env[k] = v
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "layer_profile.py")], env=env,
                         capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        raise SystemExit(out.stderr[-2000:])
    rows = {}
    for line in out.stdout.splitlines()[1:]:
        parts = line.rsplit(None, 2)
        if len(parts) == 3:
            try:
                rows[parts[0].replace(" x3", "").strip()] = float(parts[1])
            except ValueError:
                pass
        elif line.startswith("total"):
            rows["total conv kernels"] = float(line.split()[-1])
    return rows


def main():
    builds = [a.split("=", 1) for a in sys.argv[1:]]
    res = {name: run(lib) for name, lib in builds}
    keys = sorted(res[builds[0][0]], key=lambda k: -res[builds[0][0]][k])
    print(f"{'tag':58s}" + "".join(f"{n:>10s}" for n, _ in builds))
    for k in keys:
        print(f"{k:58s}" + "".join(f"{res[n].get(k, float('nan')):10.3f}" for n, _ in builds))


if __name__ == "__main__":
    main()
