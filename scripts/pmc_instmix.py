#!/usr/bin/env python3
"""Reduce rocprofv3 SQ counter passes to an instruction mix per launch.

usage: pmc_instmix.py KERNEL_SUBSTRING OUT.json DIR [DIR ...]
Each DIR holds one `rocprofv3 --pmc <up to 8 SQ counters>` pass in CSV form
(scripts/profile_instmix.sh).  Values are medians over the matching
dispatches of the per-dispatch sums.  Units (MI355X_MICROARCH.md, SQ PMC
table): SQ_WAVE_CYCLES, SQ_WAIT_* and SQ_ACTIVE_INST_* count quad-cycles;
SQ_INSTS_* count wave instructions; SQ_THREAD_CYCLES_VALU counts cycles x
active lanes of VALU instructions.
"""
import csv
import glob
import json
import os
import statistics
import sys


def collect(kernel, d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if kernel not in row.get("Kernel_Name", ""):
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            c = per.setdefault(row["Counter_Name"], {})
            c[key] = c.get(key, 0.0) + float(row["Counter_Value"])
    return {name: statistics.median(v.values()) for name, v in per.items() if v}


def main():
    kernel, out, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    m = {}
    for d in dirs:
        m.update(collect(kernel, d))
    if not m:
        raise SystemExit(f"no rows for {kernel} under {dirs}")
    g = m.get
    derived = {}
    if g("SQ_INSTS_VALU") and g("SQ_WAVES"):
        derived["valu_insts_per_wave"] = g("SQ_INSTS_VALU") / g("SQ_WAVES")
    tot = sum(g(k, 0) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH",
                                "SQ_INSTS_VMEM"))
    if tot:
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM"):
            if g(k) is not None:
                derived["share_" + k[9:].lower()] = g(k) / tot
    if g("SQ_THREAD_CYCLES_VALU") and g("SQ_ACTIVE_INST_VALU"):
        # mean active lanes of a VALU instruction / 64 (both counters taken in
        # the same unit: quad-cycles, resp. quad-cycles x active lanes)
        derived["valu_lane_utilisation"] = g("SQ_THREAD_CYCLES_VALU") / (64.0 * g("SQ_ACTIVE_INST_VALU"))
    if g("SQ_WAVE_CYCLES"):
        for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_WAIT_ANY"):
            if g(k) is not None:
                derived["frac_wave_cycles_" + k[3:].lower()] = g(k) / g("SQ_WAVE_CYCLES")
    if g("SQ_INSTS_VALU"):
        for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64",
                  "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT", "SQ_INSTS_VALU_FMA_F32"):
            if g(k) is not None:
                derived["valu_share_" + k[14:].lower()] = g(k) / g("SQ_INSTS_VALU")
    json.dump({"kernel": kernel, "counters_per_launch": m, "derived": derived}, open(out, "w"), indent=1)
    print(json.dumps(derived, indent=1))


if __name__ == "__main__":
    main()
