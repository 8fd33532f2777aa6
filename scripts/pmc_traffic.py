#!/usr/bin/env python3
"""Reduce rocprofv3 PMC passes to HBM bytes per launch of a config's
dominant kernel, merged into profiles/<round>_pmc_traffic.json under the
workload label bench.py prints (its roofline.traffic).

usage: pmc_traffic.py CONFIG FETCH_DIR WRITE_DIR OUT.json FRAMES [FRAMES_PER_LAUNCH]
(FRAMES_PER_LAUNCH > 1, c2/c3: the passes ran PMC_FRAMES launches of that
many frames; the entry is keyed "<workload> | B frames per launch" and
carries bytes per launch and per frame)
Each DIR holds one rocprofv3 --pmc pass (FETCH_SIZE, resp. WRITE_SIZE; they
cannot share a pass on gfx950) in CSV form over FRAMES frames of the config
(scripts/pmc_workload.py).  Corrections from
/opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE is in KiB and
reports half the bytes of wide streaming reads on gfx950 (x2 here);
WRITE_SIZE is exact for this code's store patterns (calibrated on
unpack_kernel, profiles/r02_pmc_calibration.json).
c2 / c3: the render kernel, the median over its launches.  c4 / c5: the
soft-shadow stage's kernels (wf_cone, wf_listtest, wf_widetest, wf_occlude4<soft>: the
roofline's kernels for those configs), summed over a frame's launches
(bench.py prices them per frame), and the whole frame's bytes beside it.
"""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd"), os.path.join(ROOT, "tests")]
from bench import CONFIGS, KERNELS, WAVEFRONT  # noqa: E402


def per_dispatch(d, counter):
    """[(kernel name, value)] per dispatch, in dispatch order."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            key = int(row.get("Dispatch_Id") or row.get("Correlation_Id"))
            name, v = vals.get(key, (row.get("Kernel_Name", ""), 0.0))
            vals[key] = (name, v + float(row["Counter_Value"]))
    return [vals[k] for k in sorted(vals)]


def main():
    cfg, fdir, wdir, out, frames = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5])
    fpl = int(sys.argv[6]) if len(sys.argv) > 6 else 1
    spec, W, H, SPP, label = CONFIGS[cfg][:5]
    workload = "%s %dx%d %dspp depth 50" % (label, W, H, SPP)
    if fpl > 1:
        workload += " | %d frames per launch" % fpl
    kerns = [k.strip() for k in KERNELS[cfg].replace("rtgo::", "").split("+")]  # (c4/c5: the soft-shadow stage)
    fetch = per_dispatch(fdir, "FETCH_SIZE")
    write = per_dispatch(wdir, "WRITE_SIZE")

    def pick(rows):
        return [v for n, v in rows if any(k in n for k in kerns)]

    kf, kw = pick(fetch), pick(write)
    if not kf or not kw:
        raise SystemExit(f"no {kerns} rows")
    res = {"kernel": KERNELS[cfg], "frames_profiled": frames}
    if cfg in WAVEFRONT:
        fb = sum(kf) / frames * 1024 * 2
        wb = sum(kw) / frames * 1024
        res.update({
            "unit": "per frame (the kernel's launches of one frame)",
            "launches_per_frame": len(kf) / frames,  # (all three kernels' launches)
            "fetch_bytes_corrected": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb,
            "frame_fetch_bytes_all_kernels": sum(v for _, v in fetch) / frames * 1024 * 2,
            "frame_write_bytes_all_kernels": sum(v for _, v in write) / frames * 1024,
        })
    else:
        fb = statistics.median(kf) * 1024 * 2
        wb = statistics.median(kw) * 1024
        res.update({"unit": "per launch (median)", "fetch_bytes_corrected": fb, "write_bytes": wb,
                    "hbm_bytes_per_launch": fb + wb, "algorithmic_bytes_per_launch": (W * H * 16 + 4096) * fpl,
                    "frames_per_launch": fpl, "hbm_bytes_per_frame": (fb + wb) / fpl})
    res["note"] = ("FETCH_SIZE (KiB) x1024 x2 per MI355X_MICROARCH.md §HBM (gfx950 counts half the bytes of wide "
                   "reads); WRITE_SIZE (KiB) x1024, exact for these stores (profiles/r02_pmc_calibration.json)")
    try:
        with open(out) as f:
            d = json.load(f)
    except (OSError, ValueError):
        d = {}
    d[workload] = res
    with open(out, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps({workload: res}))


if __name__ == "__main__":
    main()
