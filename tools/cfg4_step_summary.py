#!/usr/bin/env python3
"""Per-step kernel table of a rocprofv3 kernel trace (tools/gpu_cfg4prof.sh): the launches between
the last two env_step_kernel starts (one full training step: env.step, push, learn, act), grouped
into the step's phases. Usage: python tools/cfg4_step_summary.py <run_kernel_trace.csv> [title]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
title = sys.argv[2] if len(sys.argv) > 2 else "one training step"
idx = [i for i, r in enumerate(rows) if "env_step_kernel" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
t0 = int(rows[a]["Start_Timestamp"])
print(f"## {title}: kernels of one step (last two env_step_kernel starts)\n")
print("| start us | dur us | grid (threads x, y, z) | kernel |\n|---|---|---|---|")
tot = {}
for r in rows[a:b]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    tot[name] = tot.get(name, 0.0) + d
    print(f"| {(int(r['Start_Timestamp']) - t0) / 1e3:.1f} | {d:.1f} | {r['Grid_Size_X']}, {r['Grid_Size_Y']}, "
          f"{r['Grid_Size_Z']} | `{name[:70]}` |")
span = (int(rows[b]["Start_Timestamp"]) - t0) / 1e3
print(f"\nstep span {span:.1f} us; busiest kernels:\n")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:8]:
    print(f"* `{k[:70]}` {v:.1f} us ({100 * v / span:.1f} %)")
