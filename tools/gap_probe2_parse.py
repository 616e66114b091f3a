#!/usr/bin/env python3
"""Median gap (us) before each probe kernel of tools/gap_probe2.py on s1's queue; for the
waits (i-k) the gap is from the end of s2's last kernel before the record."""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
qs = {}
for r in rows:
    qs.setdefault(r["Queue_Id"], []).append(r)
order = sorted(qs, key=lambda k: -len(qs[k]))
s1, s2 = qs[order[0]], qs[order[1]]
per1, per2 = 48, 24
labels = ["a1 (after the holder)", "a2 (back to back)", "f record DisableTiming", "g record +DisableSystemFence",
          "h record +ReleaseToDevice", "i wait (DisableTiming)", "j wait (+DisableSystemFence)",
          "k wait (+ReleaseToDevice)"]
gaps = [[] for _ in labels]
n = min(len(s1) // per1, len(s2) // per2)
for it in range(3, n):
    blk = s1[it * per1:(it + 1) * per1]
    prev = blk[39]
    for i, k in enumerate(blk[40:45]):
        gaps[i].append((int(k["Start_Timestamp"]) - int(prev["End_Timestamp"])) / 1e3)
        prev = k
    b2 = s2[it * per2:(it + 1) * per2]
    for j in range(3):
        last = b2[j * 8 + 7]
        k = blk[45 + j]
        gaps[5 + j].append((int(k["Start_Timestamp"]) - int(last["End_Timestamp"])) / 1e3)
print("kernels s1", len(s1), "s2", len(s2), "iterations", n)
for i, l in enumerate(labels):
    print(f"{l:34s} median gap {statistics.median(gaps[i]):7.1f} us")
