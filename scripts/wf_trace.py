#!/usr/bin/env python3
"""Per-kernel totals and one mid-frame batch's dispatch sequence from a
rocprofv3 --kernel-trace csv (wavefront pipeline):  wf_trace.py <dir>"""
import csv
import glob
import re
import sys
from collections import defaultdict

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))


def nm(s):
    m = re.search(r"(wf_\w+|reduce_kernel|path_kernel|rocclr_\w+)", s)
    return m.group(1) if m else s[:20]


seq = [(nm(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows]
tot = defaultdict(float)
for n, d in seq:
    tot[n] += d
for n, d in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"{n:28s} {d / 1e3:10.2f} ms")
gen = [k for k, s in enumerate(seq) if s[0] == "wf_generate"]
if gen:
    i = gen[len(gen) // 2]
    j = i + 1
    while j < len(seq) and seq[j][0] != "wf_accumulate":
        j += 1
    print(" ".join(f"{n[3:6]}:{d:.0f}" for n, d in seq[i:j + 1]))
