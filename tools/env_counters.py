#!/usr/bin/env python3
"""Summary of tools/gpu_env_counters_r4.sh's passes for env_step_kernel: SQ ratios (of
SQ_WAVE_CYCLES), instructions per wave by kind, and HBM bytes per env-step from FETCH_SIZE
(doubled: gfx950 tallies a 128-B request at 64 B, /opt/skills/guides/MI355X_MICROARCH.md HBM) and
WRITE_SIZE, both KiB per dispatch, mean of the last 5 dispatches (the timed region).
Usage: env_counters.py DIR [envs [phase grid people robots]] -- the workload fields let bench.py
match the record to its own line (tools/gpu_r6_counters.sh); the effective clock comes from the
GRBM pass (GRBM_GUI_ACTIVE / 8 XCDs / duration, as tools/kstats.py)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kstats import counters, durations, traces  # noqa: E402


def env_entry(d):
    f = traces(d, "*counter_collection.csv")
    if not f:
        return {}
    for k, v in counters(f).items():
        if "env_step_kernel" in k:
            return v
    return {}


def main():
    d = sys.argv[1]
    E = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
    wl = sys.argv[3:7]
    c = {}
    for p in ("sq", "sq2", "gr", "fe", "wr"):
        c.update(env_entry(os.path.join(d, p)))
    grdur = None  # the duration in the pass that counted GRBM_GUI_ACTIVE (its own, or the SQ pass)
    gt = traces(os.path.join(d, "gr"), "*kernel_trace.csv") or traces(os.path.join(d, "sq"), "*kernel_trace.csv")
    if gt:
        for k, v in durations(gt).items():
            if "env_step_kernel" in k:
                grdur = sum(v[-5:]) / len(v[-5:])
    dur = None
    t = traces(os.path.join(d, "t"), "*kernel_trace.csv")
    if t:
        for k, v in durations(t).items():
            if "env_step_kernel" in k:
                dur = sum(v[-10:]) / len(v[-10:])
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    waves = c.get("SQ_WAVES", 0.0)
    rec = {"kernel": "env_step_kernel", "envs": E, "kernel_us_trace": dur}
    if len(wl) == 4:
        rec.update(phase=wl[0], grid=[int(wl[1]), int(wl[1])], people=int(wl[2]), robots=int(wl[3]))
    if c.get("GRBM_GUI_ACTIVE") and grdur:
        rec["clock_ghz"] = round(c["GRBM_GUI_ACTIVE"] / 8 / (grdur * 1e-6) / 1e9, 3)
    if wc:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS"):
            if n in c:
                rec[n.lower() + "_frac"] = round(c[n] / wc, 4)
    if waves:
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM"):
            if n in c:
                rec[n.lower() + "_per_wave"] = round(c[n] / waves, 1)
        rec["waves"] = waves
    if "SQ_LDS_BANK_CONFLICT" in c:
        rec["lds_bank_conflict"] = c["SQ_LDS_BANK_CONFLICT"]
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        fb, wb = c["FETCH_SIZE"] * 1024.0, c["WRITE_SIZE"] * 1024.0
        rec.update({"fetch_kib": c["FETCH_SIZE"], "write_kib": c["WRITE_SIZE"],
                    "bytes_per_launch": 2 * fb + wb, "bytes_per_env_step": (2 * fb + wb) / E,
                    "bytes_per_launch_raw": fb + wb, "bytes_per_env_step_raw": (fb + wb) / E,
                    "method": "separate --pmc FETCH_SIZE / WRITE_SIZE passes; bytes = 2*FETCH + WRITE"})
        if dur:
            rec["hbm_gbs"] = round((2 * fb + wb) / (dur * 1e-6) / 1e9, 1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
