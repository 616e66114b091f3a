#!/usr/bin/env python3
"""Median gap (us) before each probe kernel of tools/gap_probe.py on s1's queue."""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
qs = {}
for r in rows:
    qs.setdefault(r["Queue_Id"], []).append(r)
q = max(qs, key=lambda k: len(qs[k]))  # s1: 40 holders + 6 probes per iteration
seq = qs[q]
per = 46
labels = ["a1 (after the holder)", "a2 (back to back)", "b (timing event between)", "c (event between)",
          "d (wait on an old event)", "e (wait on a pending event)"]
gaps = [[] for _ in range(6)]
n = len(seq) // per
for it in range(3, n):
    blk = seq[it * per:(it + 1) * per]
    prev = blk[39]
    for i, k in enumerate(blk[40:]):
        gaps[i].append((int(k["Start_Timestamp"]) - int(prev["End_Timestamp"])) / 1e3)
        prev = k
print("queue", q, "kernels", len(seq), "iterations", n)
for i in range(6):
    print(f"{labels[i]:32s} median gap {statistics.median(gaps[i]):7.1f} us")
