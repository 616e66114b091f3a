#!/usr/bin/env python3
"""Per-kernel mean duration over the last N training steps of a rocprofv3 kernel trace (the steps
between consecutive env_step launches at the end of the trace: with bench.py --other-steps 0
--env-steps 0 --start-steps 0 --no-cpu those are the timed and instrumented training passes), so the
env_step_kernel figure is comparable with the bench line's env_step_kernel_ms (the kernel_stats.csv
average also counts the episode-phase preparation launches). Usage: step_kstats.py DIR [N]"""
import collections
import csv
import glob
import os
import sys

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
env = [i for i, r in enumerate(rows) if "env_step_kernel" in r["Kernel_Name"]]
a, b = env[-n - 1], env[-1]
dur = collections.defaultdict(list)
for r in rows[a:b]:
    dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
span = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
print(f"last {n} steps: {span / n:.1f} us per step (env launch to env launch)")
for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v) / n:9.1f} us/step  {len(v):4d} x {sum(v) / len(v):8.1f} us  {k[:90]}")
