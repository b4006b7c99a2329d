"""Per-step time by kernel category from a rocprofv3 --kernel-trace --stats run.
    python tools/trace_cats.py gpurun_out/tr_X/run_kernel_stats.csv STEPS"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2])
cats = defaultdict(lambda: [0.0, 0])
for r in rows:
    n = r["Name"]
    short = re.sub(r"\(.*", "", n).replace("void ", "").replace("ev::", "")
    key = re.sub(r"<.*", "", short)
    cats[key][0] += float(r["TotalDurationNs"]) / steps / 1e3
    cats[key][1] += int(r["Calls"]) / steps
tot = sum(v[0] for v in cats.values())
for k, (us, n) in sorted(cats.items(), key=lambda kv: -kv[1][0]):
    print(f"{us:9.1f} us/step {n:6.1f} launches  {k}")
print(f"{tot:9.1f} us/step total")
