"""Print one kernel's main-loop instruction skeleton from a device .s file (hipcc
--cuda-device-only -S): MFMAs, LDS reads/writes, waits, barriers and sched_barrier region
marks, so the placement of fragment reads relative to the MFMAs that consume them can be
checked.  Usage: python tools/asm_kernel.py FILE.s MANGLED_SUBSTRING [max_lines]"""
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
maxl = int(sys.argv[3]) if len(sys.argv) > 3 else 400
lines = open(path).read().split("\n")
start = None
for i, l in enumerate(lines):
    if re.match(r"^_ZN\S*" + re.escape(pat) + r"\S*:", l):
        start = i
        break
if start is None:
    sys.exit(f"kernel {pat} not found")
keep = re.compile(r"mfma|ds_read|ds_write|s_waitcnt|s_barrier|sched_barrier|buffer_load|^\.LBB|s_cbranch|global_load|s_setprio")
n = 0
for l in lines[start:]:
    if l.startswith("\t.section") or ".Lfunc_end" in l:
        break
    if keep.search(l):
        print(l.strip())
        n += 1
        if n >= maxl:
            break
