"""Per-kernel time per step from a rocprofv3 --kernel-trace CSV directory.

    python tools/kernel_table.py DIR STEPS [N]
"""
import collections
import csv
import glob
import os
import sys


def main():
    d, steps = sys.argv[1], int(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ev::", "")
        agg[name].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(rows, rows[1:])]
    idle = sum(g for g in gaps if 0 < g < 50_000)   # idle between back-to-back launches
    print(f"idle between launches (<50 us each): {idle / steps / 1e3:.1f} us per step")
    tot = sum(sum(v) for v in agg.values()) / steps / 1e3
    print(f"kernel time per step: {tot:.1f} us over {sum(len(v) for v in agg.values()) / steps:.0f} launches")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
        print(f"{sum(v) / steps / 1e3:9.1f} us/step {len(v) / steps:6.1f} x {sum(v) / len(v) / 1e3:8.1f} us  {k[:90]}")


if __name__ == "__main__":
    main()
