"""Side-by-side of two tools/layer_profile.py outputs (old, new): per-layer ms/step and delta.

    python tools/layer_diff.py old.txt new.txt
"""
import sys


def load(path):
    out = {}
    for line in open(path):
        parts = line.rstrip().rsplit(None, 2)
        if len(parts) == 3 and parts[0].startswith(("conv3x3", "total")):
            try:
                out[parts[0].strip()] = float(parts[1])
            except ValueError:
                pass
        elif line.startswith("total"):
            out["total"] = float(line.split()[-1])
    return out


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    keys = sorted(set(a) | set(b), key=lambda k: -max(a.get(k, 0), b.get(k, 0)))
    for k in keys:
        x, y = a.get(k), b.get(k)
        d = "" if x is None or y is None else f"{y - x:+.3f}"
        print(f"{k[:62]:62s} {x if x is not None else float('nan'):7.3f} {y if y is not None else float('nan'):7.3f} {d}")


if __name__ == "__main__":
    main()
