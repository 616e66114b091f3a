#!/usr/bin/env python3
"""Top kernels of a rocprofv3 kernel_stats.csv: name, calls, average / min / max us. Usage: kstat_csv.py FILE [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{r['Name'][:72]:72s} {int(r['Calls']):6d} avg {float(r['AverageNs'])/1e3:8.1f} "
          f"min {float(r['MinNs'])/1e3:8.1f} max {float(r['MaxNs'])/1e3:8.1f}")
