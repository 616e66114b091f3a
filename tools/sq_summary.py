#!/usr/bin/env python3
"""Average SQ counters of one kernel (default env_step_kernel) over its last launches: sq_summary.py CSV [name]."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
kname = sys.argv[2] if len(sys.argv) > 2 else "env_step_kernel"
v = collections.defaultdict(collections.OrderedDict)
for r in rows:
    if kname in r["Kernel_Name"]:
        d = v[r["Counter_Name"]]
        k = int(r["Dispatch_Id"])
        d[k] = d.get(k, 0.0) + float(r["Counter_Value"])
avg = {c: sum(list(d.values())[-5:]) / len(list(d.values())[-5:]) for c, d in v.items()}
for c, x in sorted(avg.items()):
    print(f"{c:24s} {x:16.0f}")
wc = avg.get("SQ_WAVE_CYCLES")
if wc:
    for c in ["SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"]:
        if c in avg:
            print(f"  {c} / WAVE_CYCLES = {avg[c] / wc:.1%}")
if "SQ_INSTS_VALU" in avg and "SQ_WAVES" in avg:
    print(f"  VALU instructions per wave (env-step): {avg['SQ_INSTS_VALU'] / avg['SQ_WAVES']:.0f}")
