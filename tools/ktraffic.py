#!/usr/bin/env python3
"""Per-kernel HBM traffic from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
(MI355X_MICROARCH.md, HBM section: both in KiB per dispatch; gfx950's FETCH_SIZE reports about
half the bytes of wide streaming reads, so 2 x FETCH is listed beside the raw value).
usage: ktraffic.py FETCH_DIR WRITE_DIR [top]"""
import collections
import csv
import glob
import sys


def per_kernel(d, counter):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f[0])):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in acc.items()}


fe, wr = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
top = int(sys.argv[3]) if len(sys.argv) > 3 else 12
rows = sorted(fe, key=lambda k: -(fe[k][0] + wr.get(k, (0.0, 0))[0]))[:top]
print(f"{'MB/dispatch':>11s} {'fetch':>9s} {'2xfetch':>9s} {'write':>9s} {'n':>4s}  kernel")
for k in rows:
    f, n = fe[k]
    w = wr.get(k, (float("nan"), 0))[0]
    print(f"{'':11s} {f / 1024:9.2f} {2 * f / 1024:9.2f} {w / 1024:9.2f} {n:4d}  {k[:90]}")
