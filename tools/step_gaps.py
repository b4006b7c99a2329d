"""Idle gaps inside the training steps of a rocprofv3 kernel trace (steps delimited by
adam_kernel).   python tools/step_gaps.py DIR [step index] [min gap us]"""
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 4
mg = float(sys.argv[3]) if len(sys.argv) > 3 else 5.0
path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
ad = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]


def nm(r):
    return re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("ev::", ""))[:60]


tot = []
for j in range(1, len(ad) - 1):
    seg = rows[ad[j] + 1:ad[j + 1] + 1]
    t0 = int(seg[0]["Start_Timestamp"])
    end = int(seg[0]["End_Timestamp"])
    idle = 0
    for r in seg[1:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s > end:
            idle += s - end
            if j == k and (s - end) / 1e3 >= mg:
                print(f"{(end - t0) / 1e3:8.1f} gap {(s - end) / 1e3:6.1f} us before {nm(r)} (stream {r['Stream_Id']})")
        end = max(end, e)
    tot.append(((int(seg[-1]["End_Timestamp"]) - t0) / 1e3, idle / 1e3, len(seg)))
for span, idle, n in tot:
    print(f"step span {span:8.1f} us  idle {idle:6.1f} us  launches {n}")
