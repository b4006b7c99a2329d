"""Per-kernel averages of a rocprofv3 `--pmc ... --output-format csv` pass.

    python tools/pmc_kernels.py DIR [--match conv3x3]

Prints, per kernel name: dispatches, average duration, each counter's average and, when
GRBM_GUI_ACTIVE was collected, the effective shader clock (GRBM_GUI_ACTIVE / 8 XCDs /
duration; MI355X_MICROARCH.md, DVFS) and, with SQ_VALU_MFMA_BUSY_CYCLES, the MFMA pipe
utilisation over the 1024 SIMDs at that clock.
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "").replace("ev::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)[0]
    per = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            if a.match not in k:
                continue
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k in sorted(per, key=lambda k: -sum(dur[k].values())):
        d = dur[k]
        ns = sum(d.values()) / len(d)
        cs = {c: sum(v) / len(v) for c, v in per[k].items()}
        line = f"{k:60s} n={len(d):4d} avg={ns / 1e3:9.2f}us"
        for c, v in sorted(cs.items()):
            line += f" {c}={v:.4g}"
        if "GRBM_GUI_ACTIVE" in cs:
            clk = cs["GRBM_GUI_ACTIVE"] / 8 / ns   # GHz
            line += f" clk={clk:.3f}GHz"
            if "SQ_VALU_MFMA_BUSY_CYCLES" in cs:
                line += f" mfma_util={cs['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * clk * ns):.3f}"
        print(line)


if __name__ == "__main__":
    main()
