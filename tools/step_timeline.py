#!/usr/bin/env python3
"""Per-step kernel timeline of a rocprofv3 --kernel-trace run of bench.py (train mode):
the last few step windows (env_step_kernel to env_step_kernel), busy vs idle, and
the kernels of one window with their start offsets and durations."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "env_step_kernel" in r["Kernel_Name"]]
for a, b in zip(idx[-6:-1], idx[-5:]):
    seg = rows[a:b]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    print(f"step window {(t1 - t0) / 1e3:.0f} us, kernels {len(seg)}, busy {busy / 1e3:.0f} us, idle {(t1 - t0 - busy) / 1e3:.0f} us")
agg = {}
for a, b in zip(idx[-11:-1], idx[-10:]):
    for r in rows[a:b]:
        n = r["Kernel_Name"][:60]
        agg[n] = agg.get(n, 0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / 10
print("mean per step over the last 10 windows (us):")
for n, v in sorted(agg.items(), key=lambda x: -x[1]):
    print(f"  {v:8.1f}  {n}")
# one window in detail: start / end offsets (us) and the stream of every kernel
a, b = idx[-3], idx[-2]
t0 = int(rows[a]["Start_Timestamp"])
print("one step window in detail (offsets from its env_step_kernel start, us):")
for r in rows[a - 12:b + 2]:
    s0 = (int(r["Start_Timestamp"]) - t0) / 1e3
    s1 = (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"  {s0:8.1f} {s1:8.1f}  q{r.get('Queue_Id', '?'):>3s} s{r.get('Stream_Id', '?'):>3s}  {r['Kernel_Name'][:70]}")
