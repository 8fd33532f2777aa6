#!/usr/bin/env python3
"""Render-kernel time per rt_tuning variant (dev tool): median of N renders
with the schedule cached, one frame at a time.
usage: tuning_sweep.py [scene.json W H SPP] with VARIANTS="k=v,k=v;k=v;..." """
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import rtgo  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "sphere_reflections_light_facing.json"
W, H, SPP = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (800, 600, 100)
if name == "spheres10k":
    from scene_cases import spheres10k_scene

    scene = spheres10k_scene(rtgo)
else:
    scene = rtgo.Scene.load_from_file(os.path.join(ROOT, "scenes", name))
reps = int(os.environ.get("REPS", "7"))
variants = [v for v in os.environ.get("VARIANTS", "").split(";")]
lin = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
rgba = torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda")
s = torch.cuda.Stream()
for v in variants:
    kw = {}
    for kv in filter(None, v.split(",")):
        k, x = kv.split("=")
        kw[k] = float(x) if "." in x else int(x)
    ctx = rtgo.Context(0)
    ctx.set_tuning(rtgo.default_tuning(**kw))
    ctx.set_scene(scene)
    st = rtgo.default_settings()
    st.samples = SPP
    ks = []
    for i in range(reps + 1):
        st.seed = 1 + i
        ctx.render_async(W, H, st, lin.data_ptr(), rgba.data_ptr(), s.cuda_stream)
        s.synchronize()
        if i:
            ks.append(ctx.last_kernel_seconds() * 1e3)
    ctx.close()
    print(f"{name} {W}x{H}x{SPP} [{v or 'default'}]: kernel median {statistics.median(ks):.3f} ms "
          f"(min {min(ks):.3f})", flush=True)
