#!/usr/bin/env python3
"""The timed launches of a bench.py run, read from its rocprofv3 kernel trace
(dev tool, runs here on the pulled files).

usage: batched_trace.py TRACE_DIR BENCH_JSON OUT.json

bench.py (N = 1, c2/c3) issues, in order, per context: its set-up launch,
the counting launch (render_kernel<true, ...>), the warm-up launches, the
timed launches (their frame counts are the line's `launch_frames`), then the
one-frame timing.  The timed launches are therefore the dominant kernel's
dispatches that follow the counting dispatch, after the warm-up ones.  For
them this reports each launch's duration and frames, the average per-frame
kernel time (duration / frames), and the union of their spans over the frames
(the GPU time per frame when launches overlap), beside the line's own
ms_per_step and HIP-event figures.
"""
import csv
import glob
import json
import os
import sys


def union_ns(spans):
    tot, cs, ce = 0, None, None
    for a, b in sorted(spans):
        if ce is None or a > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    return tot + (ce - cs if ce is not None else 0)


def main():
    tdir, bench_json, out = sys.argv[1:4]
    line = None
    for ln in open(bench_json):
        ln = ln.strip()
        if ln.startswith("{"):
            line = json.loads(ln)
    if line is None:
        raise SystemExit(f"no JSON line in {bench_json}")
    kname = line["roofline"]["kernel"]
    frames = line["launch_frames"]
    warm = line["warmup"]
    B = line["frames_per_launch"]
    n_warm = -(-warm // B) if warm else 0
    paths = glob.glob(os.path.join(tdir, "**", "*kernel_trace.csv"), recursive=True)
    if not paths:
        raise SystemExit(f"no kernel_trace.csv under {tdir}")
    rows = sorted(csv.DictReader(open(paths[0])), key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    counting = next(i for i, n in enumerate(names) if "render_kernel<true" in n)
    dom = [r for r in rows[counting + 1:] if kname in r["Kernel_Name"]]
    timed = dom[n_warm:n_warm + len(frames)]
    launches = []
    for r, f in zip(timed, frames):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        launches.append({"frames": f, "ms": round((e - s) / 1e6, 4), "ms_per_frame": round((e - s) / 1e6 / f, 4),
                         "grid_x": int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0), "start_ns": s, "end_ns": e})
    nfr = sum(frames)
    span = union_ns([(x["start_ns"], x["end_ns"]) for x in launches])
    first, last = min(x["start_ns"] for x in launches), max(x["end_ns"] for x in launches)
    res = {
        "kernel": kname,
        "bench_cmd_line": {k: line.get(k) for k in ("value", "steps", "warmup", "ms_per_step", "launch_frames",
                                                     "frames_per_launch", "launches_in_flight")},
        "bench_hip_events": {k: line["roofline"].get(k) for k in ("kernel_ms_frames_in_flight", "busy_ms_per_frame")},
        "timed_launches": launches,
        "avg_launch_ms_per_frame": round(sum(x["ms"] for x in launches) / nfr, 4),
        "union_ms_per_frame": round(span / 1e6 / nfr, 4),
        "first_start_to_last_end_ms_per_frame": round((last - first) / 1e6 / nfr, 4),
        "trace_file": os.path.relpath(paths[0], tdir),
    }
    res["union_over_ms_per_step"] = round(res["union_ms_per_frame"] / line["ms_per_step"], 4)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
        f.write("\n")
    print(json.dumps({k: v for k, v in res.items() if k != "timed_launches"}))


if __name__ == "__main__":
    main()
