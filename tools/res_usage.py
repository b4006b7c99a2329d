"""Summarise `hipcc -Rpass-analysis=kernel-resource-usage` remarks: one line per kernel with
VGPRs, AGPRs, scratch bytes, occupancy and LDS.  Usage: python tools/res_usage.py FILE [filter]"""
import re
import sys

cur, rows = None, []
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"),
                     ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"),
                     ("lds", r"LDS Size \[bytes/block\]: (\d+)"), ("sgpr", r"SGPRs: (\d+)")):
        m = re.search(pat, line)
        if m:
            cur[key] = int(m.group(1))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for r in rows:
    if flt in r["name"]:
        print(f"{r.get('vgpr', '?'):>4} v {r.get('agpr', '?'):>4} a {r.get('scratch', '?'):>5} scr "
              f"occ {r.get('occ', '?')}  {r['name'][:110]}")
