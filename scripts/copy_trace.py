#!/usr/bin/env python3
"""rocclr blit dispatches (copyBuffer / fillBuffer) in a rocprofv3 --kernel-trace CSV, grouped by kernel, grid and
the kernel dispatched just before each (to tell which host call issued them). Usage: copy_trace.py <trace dir>"""
import collections
import csv
import glob
import os
import sys

p = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(p)), key=lambda r: int(r["Start_Timestamp"]))
g = collections.defaultdict(list)
for i, r in enumerate(rows):
    if "copyBuffer" in r["Kernel_Name"] or "fillBuffer" in r["Kernel_Name"]:
        prev = rows[i - 1]["Kernel_Name"].split("(")[0][-48:] if i else ""
        g[(r["Kernel_Name"][:30], r["Grid_Size_X"], prev)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
    print(len(v), round(sum(v) / len(v), 1), k)
