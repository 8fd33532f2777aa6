#!/usr/bin/env python3
"""A/B timing of librtgo variants on the GPU (dev tool, not the bench contract).

usage: ab_bench.py LIB [LIB...]   each LIB is timed in its own subprocess:
  kernel ms (HIP events, median of N) on the facing / as-committed / silver
  scenes at 800x600x100spp, plus the linear image checksum so variants that
  change results are visible.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys, statistics
sys.path.insert(0, os.path.join(ROOT, "concurrent-raytracer-go_amd")); sys.path.insert(0, ROOT)
import torch, rtgo
cases = json.loads(sys.argv[1]); reps = int(sys.argv[2])
s = torch.cuda.Stream(); torch.cuda.set_stream(s)
out = {}
for name, path, w, h, spp in cases:
    ctx = rtgo.Context(0); ctx.set_scene(rtgo.Scene.load_from_file(path))
    st = rtgo.default_settings(); st.samples = spp
    lin = torch.zeros(w*h*3, dtype=torch.float32, device="cuda")
    rgba = torch.zeros(w*h*4, dtype=torch.uint8, device="cuda")
    ms = []
    for i in range(reps + 2):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); ctx.render_async(w, h, st, lin.data_ptr(), rgba.data_ptr(), s.cuda_stream); e1.record()
        torch.cuda.synchronize()
        if i >= 2: ms.append(e0.elapsed_time(e1))
    out[name] = {"ms": statistics.median(ms), "min": min(ms), "sum": float(lin.double().sum())}
    ctx.close()
print("RESULT", json.dumps(out))
'''.replace("ROOT", repr(ROOT))


def main():
    libs = sys.argv[1:]
    reps = int(os.environ.get("AB_REPS", "5"))
    sc = os.path.join(ROOT, "scenes")
    cases = [
        ("facing", os.path.join(sc, "sphere_reflections_light_facing.json"), 800, 600, 100),
        ("committed", os.path.join(sc, "sphere_reflections_light.json"), 800, 600, 100),
        ("silver_facing", os.path.join(sc, "final_silver_prism_purple_cube_facing.json"), 1200, 900, 100),
    ]
    if os.environ.get("AB_CASES"):
        keep = os.environ["AB_CASES"].split(",")
        cases = [c for c in cases if c[0] in keep]
    for spec in libs:
        # LIB[@KEY=VAL,KEY=VAL] — extra environment for this variant
        lib, _, extra = spec.partition("@")
        env = dict(os.environ, RTGO_LIB=os.path.abspath(lib))
        for kv in filter(None, extra.split(",")):
            k, _, v = kv.partition("=")
            env[k] = v
        lib = spec
        r = subprocess.run([sys.executable, "-c", CHILD, json.dumps(cases), str(reps)], env=env,
                           capture_output=True, text=True, timeout=600)
        line = [l for l in r.stdout.splitlines() if l.startswith("RESULT")]
        if r.returncode != 0 or not line:
            print(lib, "FAILED rc=%d" % r.returncode, r.stderr[-2000:])
            sys.exit(r.returncode or 1)
        res = json.loads(line[0][7:])
        print(lib, " ".join("%s=%.3fms(min %.3f, sum %.6g)" % (k, v["ms"], v["min"], v["sum"]) for k, v in res.items()),
              flush=True)


if __name__ == "__main__":
    main()
