"""Inter-kernel gap probe (run under rocprofv3 --kernel-trace): does the idle time between
two dependent launches grow with the bytes the first kernel wrote (end-of-kernel L2
write-back) or with what it read?  Prints nothing; analyse with tools/gap_probe.py --analyse DIR."""
import glob
import os
import sys

if len(sys.argv) > 2 and sys.argv[1] == "--analyse":
    import collections
    import csv
    p = glob.glob(os.path.join(sys.argv[2], "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(p)), key=lambda r: int(r["Start_Timestamp"]))
    gaps = collections.defaultdict(list)
    for a, b in zip(rows, rows[1:]):
        ka = a["Kernel_Name"].split("(")[0][-60:] + " g" + a["Grid_Size_X"]
        gaps[ka].append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
    for k, v in sorted(gaps.items()):
        if len(v) >= 10:
            v = sorted(v)
            print(f"{len(v):4d} median gap after {v[len(v) // 2]:6.2f} us  {k}")
    sys.exit(0)

import torch  # noqa: E402

dev = torch.device("cuda")
tiny = torch.zeros(1, device=dev)
for mb in (1, 4, 16, 64, 256):
    n = mb * (1 << 20) // 4
    buf = torch.empty(n, device=dev)
    src = torch.randn(n, device=dev)
    out = torch.empty(1, device=dev)
    for _ in range(20):
        buf.fill_(1.0)          # writes mb MiB
        tiny.add_(1.0)
    for _ in range(20):
        torch.sum(src, dim=0, out=out.view(()))   # reads mb MiB, writes 4 B
        tiny.add_(1.0)
    torch.cuda.synchronize()
