#!/usr/bin/env python3
"""Summarise a tools/profile_r2.sh output directory into profiles/<round>/.

Usage: python tools/parse_prof_r2.py gpurun_out/prof_<tag> profiles/r2 <tag>

Writes
  <dst>/summary_<tag>.md         kernel stats of each phase's timed region, the bench line,
                                 the env_step_kernel HBM traffic from the PMC passes
  <dst>/env_traffic_<phase>.json traffic record bench.py reads (roofline.traffic)
  <dst>/bench_<tag>.json         the bench line of the driver's command
  <dst>/kernel_stats_<tag>_<phase>.csv  rocprofv3 --stats output as collected

HBM bytes follow MI355X_MICROARCH.md's HBM/rocprofv3 section: FETCH_SIZE and WRITE_SIZE
are KiB per dispatch; on gfx950 FETCH_SIZE under-reports wide coalesced streaming reads by
2x, so the line carries both the raw sum (FETCH + WRITE) and the corrected one (2 FETCH +
WRITE, an upper bound for this kernel's mix of narrow gathers and streaming loads).
The profiled runs switch the bench's extras off, so the last `steps` launches of every
kernel are the timed region.
"""
import collections
import csv
import json
import os
import shutil
import sys


def trace(path):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        per[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return per


def pmc(path, counter, kernel_sub="env_step_kernel"):
    vals = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if kernel_sub in r["Kernel_Name"] and r["Counter_Name"] == counter:
            d = int(r["Dispatch_Id"])
            vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def bench_line(path):
    if not os.path.exists(path):
        return None
    lines = [l for l in open(path) if l.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def short(name, n=80):
    return name if len(name) <= n else name[:n] + "..."


def main():
    src, dst, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    os.makedirs(dst, exist_ok=True)
    out = [f"# rocprofv3 summary `{tag}`", "",
           "Commands: `tools/profile_r2.sh` -- `bench.py --steps 20 --warmup 5` (the driver's command) and, per "
           "episode phase, `rocprofv3 --kernel-trace --stats` / `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` of "
           "`bench.py --steps 20 --warmup 5 --no-cpu --other-steps 0 --env-steps 0 --start-steps 0 --phase <phase>` "
           "(cfg3: 128x128, P=2276, R=16, the bench's envs per GPU (bench line), strict schedule, f32 Q-net).", ""]
    b = bench_line(os.path.join(src, "bench.json"))
    if b:
        shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, f"bench_{tag}.json"))
        out += ["## bench line (driver command)", "",
                f"* value {b['value'] / 1e6:.3f} M env-steps/s ({b['schedule'] if 'schedule' in b else b['config']['schedule']}), "
                f"ms/step {b['ms_per_step']:.3f}, env_step_kernel {b['env_step_kernel_ms'] * 1e3:.1f} us, "
                f"roofline frac {b['roofline']['frac']:.3f}",
                f"* other schedule: {json.dumps(b.get('other_schedule'))}",
                f"* env-only: {b.get('env_only_steps_per_s', 0) / 1e6:.3f} M env-steps/s",
                f"* start phase: {json.dumps(b.get('start_phase'))}", ""]
    for phase in ("stationary", "start"):
        tdir = os.path.join(src, f"train_{phase}")
        if not os.path.isdir(tdir):
            continue
        shutil.copy(os.path.join(tdir, "run_kernel_stats.csv"), os.path.join(dst, f"kernel_stats_{tag}_{phase}.csv"))
        bl = bench_line(os.path.join(src, f"train_{phase}.log"))
        n = bl["steps"] if bl else 20
        per = trace(os.path.join(tdir, "run_kernel_trace.csv"))
        # timed region: from the first of the last n env.step launches to the end of the last
        env = sorted(per[[k for k in per if "env_step_kernel" in k][0]])
        t0, t1 = env[-n][0], env[-1][1]
        rows = []
        for k, v in per.items():
            sel = [e - s for s, e in v if s >= t0 - 1000000 and s <= t1]
            sel = [e - s for s, e in sorted(v)[-n:]] if "env_step_kernel" in k else sel
            if sel:
                rows.append((sum(sel) / len(sel), len(sel), k))
        rows.sort(key=lambda r: -r[0] * r[1])
        out += [f"## phase `{phase}`: kernels of the timed region (last {n} steps, kernel trace)", ""]
        if bl:
            out += [f"bench line of this run: {bl['value'] / 1e6:.3f} M env-steps/s, {bl['ms_per_step']:.3f} ms/step, "
                    f"HIP-event env_step_kernel {bl['env_step_kernel_ms'] * 1e3:.1f} us", ""]
        out += ["| kernel | launches | avg us |", "|---|---|---|"]
        for avg, cnt, k in rows[:16]:
            out.append(f"| `{short(k)}` | {cnt} | {avg / 1e3:.1f} |")
        out.append("")
        kern_us = sum(e - s for s, e in env[-n:]) / n / 1e3
        fp = os.path.join(src, f"fetch_{phase}", "run_counter_collection.csv")
        wp = os.path.join(src, f"write_{phase}", "run_counter_collection.csv")
        fetch = pmc(fp, "FETCH_SIZE")[-n:] if os.path.exists(fp) else []
        write = pmc(wp, "WRITE_SIZE")[-n:] if os.path.exists(wp) else []
        if fetch and write:
            E = bl["config"]["envs_per_gpu"] if bl else 4096
            f_kib, w_kib = sum(fetch) / len(fetch), sum(write) / len(write)
            raw = (f_kib + w_kib) * 1024
            corr = (2 * f_kib + w_kib) * 1024
            bpe = bl["roofline"]["bytes_per_env_step"] if bl else None
            out += [f"### env_step_kernel HBM traffic (PMC, last {len(fetch)} launches = timed region)", "",
                    f"* average duration {kern_us:.1f} us (kernel trace)",
                    f"* FETCH_SIZE {f_kib:.0f} KiB/launch, WRITE_SIZE {w_kib:.0f} KiB/launch",
                    f"* raw FETCH+WRITE {raw / 1e6:.1f} MB/launch = {raw / E:.0f} B/env-step; corrected "
                    f"2*FETCH+WRITE {corr / 1e6:.1f} MB/launch = {corr / E:.0f} B/env-step",
                    f"* algorithmic bytes (bench.py bytes_per_env_step) {bpe} B/env-step -> "
                    f"{bpe * E / (kern_us * 1e-6) / 1e9:.0f} GB/s = {bpe * E / (kern_us * 1e-6) / 8e12:.3f} of 8 TB/s"
                    if bpe else "", ""]
            json.dump({"kernel": "env_step_kernel", "phase": phase, "envs": E, "fetch_kib": f_kib, "write_kib": w_kib,
                       "bytes_per_launch_raw": raw, "bytes_per_launch": corr, "bytes_per_env_step": corr / E,
                       "bytes_per_env_step_raw": raw / E, "kernel_us_trace": kern_us, "source": tag,
                       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (KiB per dispatch), "
                                 "last launches = timed region; bytes = 2*FETCH (gfx950 correction) + WRITE"},
                      open(os.path.join(dst, f"env_traffic_{phase}.json"), "w"), indent=1)
    open(os.path.join(dst, f"summary_{tag}.md"), "w").write("\n".join(out) + "\n")
    print("\n".join(out))


if __name__ == "__main__":
    main()
