#!/usr/bin/env python3
"""Idle gaps between consecutive kernels of the training step in a rocprofv3 kernel trace: the
timeline of one step (from the act kernel before the last env_step) and the gap total per step.
Usage: step_gaps.py DIR"""
import csv
import glob
import os
import sys

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
env = [i for i, r in enumerate(rows) if "env_step_kernel" in r["Kernel_Name"]]
if len(env) < 3:
    sys.exit("fewer than 3 env_step launches in the trace")
# one step: from the kernel after env launch k-1's learn to env launch k's learn end = between two env launches
a, b = env[-3], env[-2]
t0 = int(rows[a]["Start_Timestamp"])
busy_end = t0
gap = 0
print("   start     end     dur    gap  queue kernel")
for r in rows[a:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = max(0, s - busy_end)
    gap += g
    busy_end = max(busy_end, e)
    print("%8.1f %8.1f %7.1f %6.1f  q%s  %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, g / 1e3, r["Queue_Id"],
                                              r["Kernel_Name"][:70]))
span = int(rows[b]["Start_Timestamp"]) - t0
print("step span %.1f us, idle gaps %.1f us (%.1f %%)" % (span / 1e3, gap / 1e3, 100.0 * gap / span))
# every step of the trace between consecutive env launches: span and idle gaps (host-bound steps show
# up as gaps here even when the one printed above has none)
print("all steps (env launch k -> k+1): span us / idle us")
for a, b in zip(env[:-1], env[1:]):
    t0 = int(rows[a]["Start_Timestamp"])
    busy_end, gap = t0, 0
    for r in rows[a:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap += max(0, s - busy_end)
        busy_end = max(busy_end, e)
    print("  %8.1f %7.1f" % ((int(rows[b]["Start_Timestamp"]) - t0) / 1e3, gap / 1e3))
