#!/usr/bin/env python3
"""Timeline of the last encode call in a rocprofv3 kernel trace (profiling helper, not product code):
the kernels from the last k_clear on, with start / end relative to it and their queue (the main
and the side stream of the call).   usage: trace_timeline.py DIR_OR_CSV [min_us]"""
import csv
import glob
import os
import sys

path = sys.argv[1]
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
if os.path.isdir(path):
    path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[-1]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_clear" in r["Kernel_Name"]]
last = rows[starts[-1]:] if starts else rows
t0 = int(last[0]["Start_Timestamp"])
qkey = "Queue_Id" if "Queue_Id" in last[0] else "Stream_Id"
for r in last:
    a, b = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    if (b - a) / 1e3 < min_us:
        continue
    name = r["Kernel_Name"].replace("ctok_dev::", "").split("(")[0]
    print("%-46s q%-3s %9.1f -> %9.1f  (%8.1f us)" % (name[:46], r.get(qkey, "?"), a / 1e3, b / 1e3, (b - a) / 1e3))
end = max(int(r["End_Timestamp"]) for r in last) - t0
print("call span %.1f us" % (end / 1e3))
