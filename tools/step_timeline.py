#!/usr/bin/env python3
"""Print the last N kernel records of a rocprofv3 kernel trace in start order (start, end, duration
in us relative to the first printed record, queue id, kernel name). Usage: step_timeline.py DIR [N]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))[-n:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print("%9.1f %9.1f %7.1f  q%s  %s" % (s / 1e3, e / 1e3, (e - s) / 1e3, r["Queue_Id"], r["Kernel_Name"][:80]))
