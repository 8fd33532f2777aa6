#!/usr/bin/env python3
"""Summarize scripts/cli_trace.sh output dirs (dev tool, runs here).

usage: cli_trace_summary.py OUT.json LABEL=gpurun_out/cli_trace_TAG [LABEL=DIR ...]
Per dir: the three fresh-process runs' benchmark_data (Render time and its
breakdown, process wall time) and, from the rocprofv3 run, the HIP calls
over 0.1 ms, the render-path kernels and the copies on one time axis (ms
from the first traced call).
"""
import csv
import glob
import json
import os
import sys


def summarize(d):
    out = {"runs": []}
    for f in sorted(glob.glob(os.path.join(d, "run[0-9].json"))):
        b = json.load(open(f))
        out["runs"].append({k: b.get(k) for k in ("render_time_seconds", "kernel_time_seconds", "rays_per_second",
                                                  "render_breakdown_seconds", "setup_time", "process_wall_s")})
    tr = os.path.join(d, "trace")
    api = glob.glob(os.path.join(tr, "*hip_api_trace.csv"))
    if api:
        rows = list(csv.DictReader(open(api[0])))
        t0 = min(int(r["Start_Timestamp"]) for r in rows)
        ev = []
        for r in rows:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if (e - s) > 100_000:
                ev.append((s, "api", r["Function"], e - s))
        for f, kind, key in (("kernel_trace", "kernel", "Kernel_Name"), ("memory_copy_trace", "copy", "Direction")):
            for p in glob.glob(os.path.join(tr, f"*{f}.csv")):
                for r in csv.DictReader(open(p)):
                    name = r.get(key, "")
                    if kind == "kernel" and not any(x in name for x in ("render_kernel", "warm", "sched_blocks")):
                        continue
                    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                    ev.append((s, kind, name[:70], e - s))
        ev.sort()
        out["timeline_ms"] = [[round((s - t0) / 1e6, 3), kind, name, round(dur / 1e6, 3)] for s, kind, name, dur in ev]
    return out


def main():
    res = {"note": "scripts/cli_trace.sh: `raytracer scenes/sphere_reflections_light_facing.json out.png 800 600` "
                   "in fresh processes on one MI355X; timeline = [ms, kind, name, duration ms]"}
    for arg in sys.argv[2:]:
        label, _, d = arg.partition("=")
        res[label] = summarize(d)
    with open(sys.argv[1], "w") as f:
        json.dump(res, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
