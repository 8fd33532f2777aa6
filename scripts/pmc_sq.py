#!/usr/bin/env python3
"""Per-dispatch SQ counter summary of the render kernel (dev tool).

usage: pmc_sq.py DIR [KERNEL_SUBSTRING]
DIR holds one rocprofv3 --pmc pass in CSV form.  Prints, per counter, the
median over dispatches, and the derived per-wave figures (SQ cycle counters
count quad-cycles on gfx950, MI355X_MICROARCH.md).
"""
import collections
import csv
import glob
import os
import statistics
import sys

d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "render_kernel<false, true, false>"
vals = collections.defaultdict(dict)
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if kern not in row.get("Kernel_Name", ""):
            continue
        key = row.get("Dispatch_Id") or row.get("Correlation_Id")
        c = row["Counter_Name"]
        vals[c][key] = vals[c].get(key, 0.0) + float(row["Counter_Value"])
med = {c: statistics.median(v.values()) for c, v in vals.items()}
for c in sorted(med):
    print(f"{c:28s} {med[c]:.4g}")
w = med.get("SQ_WAVES")
if w:
    for c in ("SQ_WAVE_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY",
              "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_INSTS_LDS", "SQ_INSTS_VMEM"):
        if c in med:
            print(f"per wave {c:28s} {med[c] / w:.4g}")
    if "SQ_WAVE_CYCLES" in med and "SQ_INSTS_VALU" in med:
        print(f"VALU instructions per wave-cycle (x4 quad): {med['SQ_INSTS_VALU'] / (4 * med['SQ_WAVE_CYCLES']):.4f}")
