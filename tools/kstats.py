#!/usr/bin/env python3
"""Per-kernel summary of a profile directory made by tools/gpu_learnprof.sh (or any run with
t/ = --kernel-trace --stats, sq/ = one --pmc pass of SQ counters, gr/ = GRBM_GUI_ACTIVE):
mean duration of the last launches, SQ counter ratios, MFMA busy fraction and the effective
clock (GRBM_GUI_ACTIVE / 8 XCDs / duration). Usage: kstats.py DIR [min_us]"""
import collections
import csv
import glob
import os
import sys


def traces(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return f[0] if f else None


def durations(path):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        per[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return per


def counters(path):
    v = collections.defaultdict(lambda: collections.defaultdict(collections.OrderedDict))
    for r in csv.DictReader(open(path)):
        d = v[r["Kernel_Name"]][r["Counter_Name"]]
        k = int(r["Dispatch_Id"])
        d[k] = d.get(k, 0.0) + float(r["Counter_Value"])
    out = {}
    for kn, cs in v.items():
        out[kn] = {c: sum(list(d.values())[-5:]) / len(list(d.values())[-5:]) for c, d in cs.items()}
    return out


def main():
    d = sys.argv[1]
    min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
    t = traces(os.path.join(d, "t"), "*kernel_trace.csv")
    per = durations(t) if t else {}
    sqf = traces(os.path.join(d, "sq"), "*counter_collection.csv")
    sq = counters(sqf) if sqf else {}
    grf = traces(os.path.join(d, "gr"), "*counter_collection.csv")
    gr = counters(grf) if grf else {}
    grt = traces(os.path.join(d, "gr"), "*kernel_trace.csv")
    grdur = durations(grt) if grt else {}
    rows = []
    for k, v in per.items():
        tail = v[-10:]
        rows.append((sum(tail) / len(tail), len(v), k))
    for us, n, k in sorted(rows, reverse=True):
        if us < min_us:
            continue
        line = f"{us:9.1f} us x{n:4d}  {k[:70]}"
        c = sq.get(k)
        if c and c.get("SQ_WAVE_CYCLES"):
            wc = c["SQ_WAVE_CYCLES"]
            line += (f" | wait {c.get('SQ_WAIT_ANY', 0) / wc:5.1%} instwait {c.get('SQ_WAIT_INST_ANY', 0) / wc:5.1%}"
                     f" active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.1%} lds {c.get('SQ_ACTIVE_INST_LDS', 0) / wc:5.1%}"
                     f" bankconf {c.get('SQ_LDS_BANK_CONFLICT', 0):.3g}")
            g = gr.get(k, {}).get("GRBM_GUI_ACTIVE")
            gd = grdur.get(k)
            if g and gd:
                dur = sum(gd[-5:]) / len(gd[-5:]) * 1e-6
                clk = g / 8 / dur
                if not 1.0e9 <= clk <= 2.6e9:  # GRBM_GUI_ACTIVE is chip-wide: short kernels see others' cycles
                    clk = 2.4e9  # MI355X peak engine clock
                mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
                # MFMA busy cycles summed over SIMDs: fraction of 1024 SIMDs x the kernel's cycles
                line += f" clk {clk / 1e9:4.2f} GHz mfma {mf / (1024 * clk * dur):5.1%}"
                # SQ_WAVE_CYCLES counts quad-cycles on gfx950 (x4: the mean waves resident per CU,
                # cross-checked against the env kernel's stamp-measured 7.95 per CU)
                line += f" waves/CU {4 * wc / (256 * clk * dur):5.2f}"
        print(line)


if __name__ == "__main__":
    main()
