#!/usr/bin/env python3
"""Summarise a tools/profile_run.sh output directory into a markdown file under profiles/.

HBM traffic per env_step_kernel launch from the PMC passes, following
MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so the
corrected read bytes are 2 x FETCH_SIZE (an upper bound for this kernel's mix of
narrow gathers and streaming loads; both raw and corrected values are listed).
"""
import collections
import csv
import os
import sys


def kstats(path):
    rows = list(csv.DictReader(open(path)))
    return [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]), float(r["Percentage"]))
            for r in rows]


def pmc(dirpath, counter, kernel_sub="env_step_kernel", last=None):
    rows = list(csv.DictReader(open(os.path.join(dirpath, "run_counter_collection.csv"))))
    vals = collections.OrderedDict()
    for r in rows:
        if kernel_sub in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[int(r["Dispatch_Id"])] = vals.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    v = list(vals.values())
    if last:
        v = v[-last:]
    return (sum(v) / len(v) if v else float("nan")), len(v)


def main():
    src, tag = sys.argv[1], sys.argv[2]
    out = [f"# rocprofv3 summary `{tag}`", "",
           "Command: `tools/profile_run.sh` (bench.py cfg3: 128x128, P=2276, R=16, 4096 envs, staggered warm-up 1300)", ""]
    for sect in ["train", "env"]:
        p = os.path.join(src, sect, "run_kernel_stats.csv")
        if not os.path.exists(p):
            continue
        out += [f"## kernel stats: {sect} mode", "", "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
        for name, calls, tot, avg, pct in kstats(p)[:14]:
            out.append(f"| `{name[:90]}` | {calls} | {tot / 1e6:.2f} | {avg / 1e3:.1f} | {pct:.1f} |")
        out.append("")
        # the timed region = the last `steps` launches (the stats above include the warm-up)
        log = os.path.join(src, f"{sect}.log")
        line = [l for l in open(log) if l.startswith("{")] if os.path.exists(log) else []
        if line:
            import json
            b = json.loads(line[-1])
            n = b["steps"]
            tr = list(csv.DictReader(open(os.path.join(src, sect, "run_kernel_trace.csv"))))
            per = collections.defaultdict(list)
            for r in tr:
                per[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            out += [f"Timed region (last {n} launches per kernel, from the kernel trace) vs bench.py's HIP-event "
                    f"env_step_kernel time {b['env_step_kernel_ms'] * 1e3:.1f} us:", "",
                    "| kernel | avg us (timed region) |", "|---|---|"]
            for name, *_ in kstats(p)[:8]:
                d = per[name][-n:]
                out.append(f"| `{name[:90]}` | {sum(d) / len(d) / 1e3:.1f} |")
            out.append("")
    fetch, nf = pmc(os.path.join(src, "fetch"), "FETCH_SIZE", last=10)
    write, nw = pmc(os.path.join(src, "write"), "WRITE_SIZE", last=10)
    out += ["## HBM traffic of env_step_kernel (PMC, last 10 launches of the timed region)", "",
            f"* FETCH_SIZE {fetch:.0f} KiB/launch raw ({nf} launches) -> corrected x2: {2 * fetch / 1024:.1f} MiB",
            f"* WRITE_SIZE {write:.0f} KiB/launch ({nw} launches) = {write / 1024:.1f} MiB",
            f"* traffic per launch (corrected): {(2 * fetch + write) * 1024 / 1e6:.1f} MB; "
            f"per env-step: {(2 * fetch + write) * 1024 / 4096:.0f} B", ""]
    dst = os.path.join("profiles", f"{tag}.md")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    open(dst, "w").write("\n".join(out) + "\n")
    if fetch == fetch and write == write:  # not NaN: traffic record read by bench.py
        import json
        envs = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
        json.dump({"kernel": "env_step_kernel", "envs_per_launch": envs, "fetch_kib_raw": fetch,
                   "write_kib": write, "bytes_per_launch": (2 * fetch + write) * 1024,
                   "bytes_per_env_step": (2 * fetch + write) * 1024 / envs,
                   "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes, KiB, "
                             "FETCH doubled (gfx950 streaming-read correction, MI355X_MICROARCH.md)",
                   "source": dst}, open(os.path.join(os.path.dirname(dst), "env_traffic.json"), "w"), indent=1)
    print("\n".join(out))


if __name__ == "__main__":
    main()
