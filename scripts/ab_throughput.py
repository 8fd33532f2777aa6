#!/usr/bin/env python3
"""A/B throughput of librtgo variants (dev tool, not the bench contract).

usage: ab_throughput.py [--rounds R] [--config c2] [--steps K] LIB[@KEY=VAL,...] ...
Each LIB runs `bench.py --config CFG --steps K --warmup 5 --no-cpu-baseline
--no-e2e` in its own process (RTGO_LIB=LIB), R rounds interleaved, and the
line's value, ms_per_step, one-frame kernel ms and oracle check are printed
per run and as medians per variant.  Experiment variants that change the
image (timing bounds) show check_equals_oracle false.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--steps", type=int, default=100)
    args = ap.parse_args()
    res = {spec: [] for spec in args.libs}
    for rnd in range(args.rounds):
        for spec in args.libs:
            lib, _, extra = spec.partition("@")
            env = dict(os.environ, RTGO_LIB=os.path.abspath(lib))
            for kv in filter(None, extra.split(",")):
                k, _, v = kv.partition("=")
                env[k] = v
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", args.config, "--steps", str(args.steps),
                   "--warmup", "5", "--no-cpu-baseline", "--no-e2e"]
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
            line = next((json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")), None)
            if line is None:
                print(spec, "FAILED", p.returncode, p.stderr[-1500:], flush=True)
                continue
            r = {"value": line["value"], "ms_per_step": line["ms_per_step"],
                 "kernel_ms_1": line["one_frame_in_flight"]["kernel_ms"],
                 "check_equals_oracle": line.get("check_equals_oracle")}
            res[spec].append(r)
            print(rnd, spec, json.dumps(r), flush=True)
    summary = {spec: {"value_median": statistics.median([r["value"] for r in rs]),
                      "kernel_ms_1_median": statistics.median([r["kernel_ms_1"] for r in rs])}
               for spec, rs in res.items() if rs}
    print("SUMMARY", json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
